/*
 * gcmx.h -- C-ABI of the MI355X grid-characteristic stage path.
 *
 * This is the drop-in boundary for libgcm's cubic stage loop.  Each entry point
 * names the reference interface it replaces (paths relative to
 * /root/reference/src/libgcm).  Plain C: no exceptions cross the ABI, every call
 * returns a gcmx_status and gcmx_last_error() holds the message of the last
 * failure on the calling thread (the reference throws gcm::Exception from
 * assert_* / THROW_* instead: util/infrastructure/Assertion.hpp).
 *
 * Ownership: a gcmx_ctx owns every device buffer of one body (one CubicGrid
 * mesh, or one X-slab of it on one GPU).  Threading: one host thread drives one
 * context at a time; all work of a context is issued on its own HIP stream.
 *
 * Host-side arrays passed through this ABI use the reference's DefaultMesh
 * storage order: M doubles per node, over ALL nodes including borderSize ghost
 * layers, indexed by CubicGrid::getIndex (grid/cubic/CubicGrid.hpp:141-147;
 * X slowest, last axis fastest).  On the device the context keeps its own
 * ghost-padded SoA layout.
 */
#ifndef GCMX_H
#define GCMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCMX_ABI_VERSION 3

typedef enum gcmx_status {
	GCMX_OK = 0,
	GCMX_ERR_INVALID_ARG = 1, /* reference: assert_* on arguments                     */
	GCMX_ERR_CFL = 2,         /* reference: assert_le(k, src.size()-1) in minMaxInterpolate
	                             (interpolation/EqualDistanceLineInterpolator.hpp:22-23) */
	GCMX_ERR_HIP = 3,         /* a HIP runtime call failed                            */
	GCMX_ERR_OOM = 4,         /* device allocation failed                             */
	GCMX_ERR_STATE = 5,       /* call order violated (e.g. stage before materials)    */
	GCMX_ERR_UNSUPPORTED = 6, /* configuration outside what this build implements     */
	GCMX_ERR_COMM = 7         /* RCCL error in the halo exchange                      */
} gcmx_status;

typedef struct gcmx_ctx gcmx_ctx;

/* CubicGrid<D>::ConstructionPack (grid/cubic/CubicGrid.hpp:96-101). */
typedef struct gcmx_grid_desc {
	int dim;          /* 1, 2 or 3 (Task::globalSettings.dimensionality)            */
	int border_size;  /* ghost layers, 1..8 (Task::CubicGrid::borderSize)          */
	int sizes[3];     /* inner nodes per axis; entries >= dim are ignored          */
	int start[3];     /* global index of the first inner node (CubicGrid::start)   */
	double h[3];      /* spatial steps (CubicGrid::h)                              */
} gcmx_grid_desc;

/* Which kernels gcmx_step may use (gcmx_set_kernel_path). */
typedef enum gcmx_path {
	GCMX_PATH_AUTO = 0,    /* fastest path the configuration admits                */
	GCMX_PATH_GENERIC = 1, /* one thread per node, any D / borderSize / materials  */
	GCMX_PATH_SPLIT = 2,   /* per-axis tuned kernels (march / LDS line), 3-D only  */
	GCMX_PATH_FUSED = 3    /* the whole step in one pass (k_fused_xyz), 3-D only  */
} gcmx_path;

/* Floating-point build of the one-pass step (gcmx_set_fp_mode). */
typedef enum gcmx_fp_mode {
	GCMX_FP_FMA = 0,   /* multiply-adds contracted (default): within the north-star fp64
	                      tolerance of the reference (relative L2 <= 1e-10; measured
	                      ~1e-16 per step), 6-7 % faster at 512^3                    */
	GCMX_FP_EXACT = 1  /* the reference's separate multiply and add roundings: bitwise
	                      equal to the oracle / reference CPU path                  */
} gcmx_fp_mode;

/* How gcmx_step issues the fused pass (gcmx_set_step_schedule). */
typedef enum gcmx_schedule {
	GCMX_SCHED_AUTO = 0,   /* boundary-first schedule when a halo exchange is
	                          configured, else one launch                        */
	GCMX_SCHED_SINGLE = 1, /* halo (if any) first, then one launch over all planes */
	GCMX_SCHED_XSLAB = 2,  /* interior planes on a low-priority stream beside the
	                          boundary planes, the next halo posted before the
	                          interior joins; needs X >= 4*bs     */
	GCMX_SCHED_BFIRST = 3  /* boundary planes first (thin blocks, alone on the
	                          GPU), the next halo posted, then the interior on
	                          the same stream; needs X >= 4*bs    */
} gcmx_schedule;

/* ---- library ------------------------------------------------------------ */
int         gcmx_abi_version(void);
const char* gcmx_last_error(void);
int         gcmx_pde_size(int dim); /* VelocitySigmaVariables<D>: D + D(D+1)/2 */
const char* gcmx_status_string(gcmx_status s);

/* ---- lifetime --------------------------------------------------------------
 * Replaces: AbstractFactory::createMesh + DefaultMesh ctor/allocate
 * (engine/cubic/AbstractFactory.hpp:74-79, engine/cubic/DefaultMesh.hpp:159-167)
 * and CubicGrid ctor assertions (grid/cubic/CubicGrid.hpp:184-199).
 * Allocates two zero-filled time layers on `device`. */
gcmx_status gcmx_create(const gcmx_grid_desc* desc, int device, gcmx_ctx** out);
void        gcmx_destroy(gcmx_ctx* ctx);

/* ---- set-up ----------------------------------------------------------------
 * Replaces the per-node GcmMatrices shared_ptr table DefaultMesh::gcmMatrices
 * (DefaultMesh.hpp:144) filled by MaterialsCondition::apply
 * (util/task/MaterialsCondition.hpp:23-36).  U/U1: [n_mat][dim][M*M] row-major,
 * L: [n_mat][dim][M] (GcmMatrices<M,D>::GcmMatrix {U, U1, L},
 * util/math/GridCharacteristicMethod.hpp:40-52).  n_mat in 1..255. */
gcmx_status gcmx_set_materials(gcmx_ctx* ctx, int n_mat, const double* U,
                               const double* U1, const double* L);
/* One byte per node of the all-nodes array (getIndex order); NULL means every
 * node uses material 0.  Ghost entries are ignored.  With per-node ids the 3-D
 * step runs in one pass for up to 32 materials (their tables held in LDS, and
 * floor(q) = 0 with equal axes per material); more take the per-stage path. */
gcmx_status gcmx_set_material_ids(gcmx_ctx* ctx, const uint8_t* ids_all_nodes);

/* Whole current time layer, host <-> device (DefaultMesh::pdeVariables). */
gcmx_status gcmx_upload(gcmx_ctx* ctx, const double* aos_all_nodes);
gcmx_status gcmx_download(gcmx_ctx* ctx, double* aos_all_nodes);
/* "parity-random" field: every inner component uniform in
 * [-1,1) from SplitMix64(seed), indexed in global (x,y,z,c) order of a global
 * box of `global_sizes` nodes; ghosts untouched.  Generated on the device. */
gcmx_status gcmx_fill_random(gcmx_ctx* ctx, const int global_sizes[3], uint64_t seed);

/* ---- the hot path ------------------------------------------------------------
 * gcmx_stage replaces GridCharacteristicMethodBase::stage(s, timeStep, mesh)
 * (engine/cubic/GridCharacteristicMethod.hpp:13-17, impl :42-52) followed by
 * AbstractMesh::swapCurrAndNextPdeTimeLayer(0) (engine/cubic/DefaultMesh.hpp:134-137),
 * i.e. one iteration of the stage loop body in cubic::Engine::nextTimeStep
 * (engine/cubic/Engine.cpp:108-112).  Validates Courant (floor(q) < borderSize
 * for every material/eigenvalue) where the reference would assert.
 * Asynchronous on the context stream. */
gcmx_status gcmx_stage(gcmx_ctx* ctx, int axis, double tau);
/* All `dim` stages of one time step with no border or contact work between
 * them (cubic::Engine::nextTimeStep, Engine.cpp:90-121, for a body without
 * border conditions, contacts or ODEs).  May run fused kernels; results are
 * identical to dim consecutive gcmx_stage calls.  3-D: the one-pass step
 * (k_step_tx2 / k_fused_xyz); 2-D: the one-pass step k_step2d_iso / k_step2d
 * with one material, untouched ghosts and no X-slab exchange (else the
 * per-stage kernels); 1-D: the one stage. */
gcmx_status gcmx_step(gcmx_ctx* ctx, double tau);
gcmx_status gcmx_set_kernel_path(gcmx_ctx* ctx, gcmx_path path);
/* Step schedule of the fused path and the fused kernel's y rows per block
 * (0 = automatic).  Results do not depend on either (tests/test_gpu_parity.py);
 * only the overlap of the X-slab halo exchange with compute does. */
gcmx_status gcmx_set_step_schedule(gcmx_ctx* ctx, gcmx_schedule sched, int rows_per_block);
/* The one-pass step's floating-point build (k_step_tx2 / k_fused_xyz; the
 * per-stage kernels always keep the reference's roundings).  Default FMA;
 * environment GCMX_FP=exact makes EXACT the default of new contexts. */
gcmx_status gcmx_set_fp_mode(gcmx_ctx* ctx, gcmx_fp_mode mode);
gcmx_status gcmx_get_fp_mode(const gcmx_ctx* ctx, gcmx_fp_mode* mode);
/* Which path gcmx_step would take now (after materials are set). */
gcmx_path   gcmx_effective_path(gcmx_ctx* ctx);
/* The path the last gcmx_step / gcmx_step_faces / gcmx_stage ran
 * (GCMX_PATH_AUTO before the first). */
gcmx_path   gcmx_last_step_path(gcmx_ctx* ctx);

/* ---- sibling plugin points ----------------------------------------------------
 * Replaces cubic::BorderConditions::handleBorderPoint
 * (engine/cubic/BorderConditions.hpp:94-114) for one condition on one face:
 * for each listed face node and a = 1..borderSize,
 *   ghost(-a) = inner(+a); then for each quantity q in order,
 *   q(ghost) = -q(inner) + 2 * value_q.
 * `face_nodes`: n_nodes inner multi-indices (dim ints each) on the face
 * sizes[axis]-1 (side = +1, innerSign -1) or 0 (side = -1, innerSign +1).
 * `quantities`: codes of PhysicalQuantities::T (util/Enum.hpp:27-50):
 *   2..4 = Vx..Vz, 5..10 = Sxx,Sxy,Sxz,Syy,Syz,Szz, 12 = PRESSURE.
 * `values`: the time dependency already evaluated at Clock::Time(). */
gcmx_status gcmx_border_fill(gcmx_ctx* ctx, int axis, int side, int n_nodes,
                             const int* face_nodes, int n_quantities,
                             const int* quantities, const double* values);
/* The same with the face-node list uploaded ONCE (BorderConditions' constructor
 * collects the nodes, BorderConditions.hpp:46-78; apply() reuses them every
 * stage, :81-91): gcmx_border_nodes_create copies the list to the device;
 * gcmx_border_apply enqueues the fill on the context stream with the quantities
 * passed by value (at most GCMX_MAX_BORDER_Q) -- no host synchronisation, no
 * copies per call.  A node list belongs to the context it was created on. */
#define GCMX_MAX_BORDER_Q 16
typedef struct gcmx_border_nodes gcmx_border_nodes;
gcmx_status gcmx_border_nodes_create(gcmx_ctx* ctx, int axis, int side, int n_nodes,
                                     const int* face_nodes, gcmx_border_nodes** out);
gcmx_status gcmx_border_apply(gcmx_ctx* ctx, const gcmx_border_nodes* nodes, int n_quantities,
                              const int* quantities, const double* values);
void        gcmx_border_nodes_destroy(gcmx_border_nodes* nodes);

/* One time step of a body whose cubic border conditions are UNIFORM on each face
 * (every node of the face has the same last-applying condition, or none):
 * equivalent to, for stage s = 0..dim-1, BorderConditions::apply(mesh, s) on the
 * faces of axis s (BorderConditions.hpp:81-114) followed by gcmx_stage(s)
 * (Engine::nextTimeStep, Engine.cpp:90-121, for a body without contacts).
 * faces[2*axis + (side > 0 ? 1 : 0)], 2*dim entries; quantities as in
 * gcmx_border_fill, values evaluated at Clock::Time().  In 3-D this keeps the
 * one-pass step (ghost rows and columns of the intermediate stages formed in
 * registers / LDS, x faces filled in memory first) when borderSize <= 2,
 * Z <= 512, Y, Z >= 2*borderSize + 2 and no y/z face sets PRESSURE; otherwise it
 * runs the stages with device-side face fills.  Results are identical either way. */
typedef struct gcmx_face {
	int    enabled;                       /* 0: no condition on this face      */
	int    n_quantities;                  /* <= GCMX_MAX_BORDER_Q              */
	int    quantities[GCMX_MAX_BORDER_Q]; /* PhysicalQuantities codes, in order */
	double values[GCMX_MAX_BORDER_Q];     /* timeDependency(Clock::Time())      */
} gcmx_face;
gcmx_status gcmx_step_faces(gcmx_ctx* ctx, double tau, const gcmx_face* faces);

/* PARTIAL faces (a condition's area covers part of a face, e.g. the titan
 * preset's cylinder, launcher/ndi.hpp:309-315): one byte per face node, the
 * index of the LAST condition whose area holds the node (BorderConditions::apply
 * runs the conditions in order and a later one rewrites the whole ghost,
 * BorderConditions.hpp:81-114), or GCMX_NO_FACE_CONDITION where none does (the
 * reference never writes those ghosts).  node_condition[f], f = 2*axis + (side >
 * 0), covers the face's inner nodes with the other axes in increasing order,
 * the last fastest (y faces [x][z], z faces [x][y], x faces [y][z]); NULL = no
 * condition on that face.  The maps are uploaded once (a body's border nodes are
 * static).  gcmx_step_face_map = for s = 0..dim-1: the conditions' fills of the
 * faces of axis s, then gcmx_stage(s) -- with conds[k] the k-th condition's
 * quantities and values at Clock::Time() (at most GCMX_MAX_FACE_CONDITIONS).  In
 * 3-D it keeps the one-pass step on the same terms as gcmx_step_faces (each face
 * node's ghost formed from its own condition inside the kernel); results are
 * identical either way. */
#define GCMX_MAX_FACE_CONDITIONS 8
#define GCMX_NO_FACE_CONDITION 255
typedef struct gcmx_face_map gcmx_face_map;
gcmx_status gcmx_face_map_create(gcmx_ctx* ctx, const uint8_t* const node_condition[6], gcmx_face_map** out);
void        gcmx_face_map_destroy(gcmx_face_map* map);
gcmx_status gcmx_step_face_map(gcmx_ctx* ctx, double tau, const gcmx_face_map* map, int n_conditions,
                               const gcmx_face* conditions);

/* Replaces ContactCopier::apply (engine/cubic/ContactConditions.hpp:56-68):
 * copy a box of `dst`'s current layer from a same-sized box of `src`'s current
 * layer (boxes as local multi-indices [min, max), may include ghosts).  Both
 * contexts must live on the same device. */
gcmx_status gcmx_copy_box(gcmx_ctx* dst, const int dst_min[3], const int dst_max[3],
                          gcmx_ctx* src, const int src_min[3]);

/* Replaces MaxwellViscosityOde<Mesh>::apply (rheology/ode/Ode.hpp:28-37), which
 * cubic::Engine::nextTimeStep runs after the stages (engine/cubic/Engine.cpp:115-119):
 * every stress component of every inner node of the current layer is multiplied
 * by exp(-tau / tau0[m]), m = the node's material (gcmx_set_material_ids).
 * `tau0`: one decay time per material set with gcmx_set_materials (n_mat of
 * them).  The factor is computed on the host with the C library's exp. */
gcmx_status gcmx_ode_maxwell(gcmx_ctx* ctx, double tau, const double* tau0, int n_mat);

/* One time step followed by the Maxwell ODE, as cubic::Engine::nextTimeStep runs
 * them (the stages, then the bodies' ODEs, Engine.cpp:90-121): identical results
 * to gcmx_step (faces == NULL) or gcmx_step_faces, then gcmx_ode_maxwell.  When
 * the step runs the one-pass kernel over one material, the factor multiplies the
 * stresses in the kernel's store epilogue (no second pass over the layer; with an
 * X-slab exchange the neighbours receive the scaled planes); otherwise the
 * separate scaling pass follows.  gcmx_last_ode_fused: 1 when the last
 * gcmx_step_ode folded the ODE into the step. */
gcmx_status gcmx_step_ode(gcmx_ctx* ctx, double tau, const gcmx_face* faces, const double* tau0,
                          int n_mat);
int         gcmx_last_ode_fused(gcmx_ctx* ctx);

/* ---- multi-GPU X-slab halo (replaces the dead MPI slab design,
 * src/test/TestMPI.cpp:33-50, 92-155, and the in-process ContactCopier for
 * bodies split along X) ---------------------------------------------------------*/
#define GCMX_UNIQUE_ID_BYTES 128
gcmx_status gcmx_comm_unique_id(uint8_t id[GCMX_UNIQUE_ID_BYTES]);
/* left/right: ranks owning the slabs at lower/higher X, or -1 at a physical
 * boundary.  Collective over `nranks` processes (one context per process).
 * In a ONE-rank communicator left/right may be 0 (the rank itself): the same
 * ncclSend/ncclRecv group then runs against itself, and RCCL matches a rank's
 * sends to itself with its receives in posting order, so the left ghost planes
 * receive the slab's first bs inner planes and the right ghost planes its last
 * bs (the RCCL transport exercised on a one-GPU box; not periodic).
 *
 * The communicator is NON-BLOCKING (ncclConfig_t blocking = 0): every host wait
 * on RCCL work -- its initialisation, the enqueue of each exchange group,
 * gcmx_sync / gcmx_download / gcmx_upload / gcmx_destroy on a stream the
 * exchange feeds -- polls ncclCommGetAsyncError under a timeout; a failure or a
 * timeout (a peer that never posts, a dead peer) aborts the communicator
 * (ncclCommAbort: RCCL's waiting kernels exit) and returns GCMX_ERR_COMM, and
 * every later exchange of the context fails with GCMX_ERR_COMM.  Replaces the
 * blocking MPI_Sendrecv_replace of the dead MPI design (src/test/TestMPI.cpp:33-50). */
typedef struct gcmx_comm_options {
	int    global_x;          /* inner nodes of the WHOLE grid along X, equal on every rank
	                             (0: unknown)                                              */
	int    channels_per_peer; /* -1: automatic, 0: RCCL's default, > 0: explicit (must be
	                             equal on every rank: both ends of a p2p connection use it) */
	int    min_ctas, max_ctas;/* ncclConfig_t minCTAs / maxCTAs; -1: 16 / 32, 0: RCCL's own */
	double timeout_s;         /* bound of host waits on RCCL work; <= 0: the environment's
	                             GCMX_COMM_TIMEOUT_SECONDS, default 60                       */
} gcmx_comm_options;
/* Channels per peer (checked contract).  Automatic (channels_per_peer = -1):
 * gcmx_comm_channels_rule of inputs every rank holds alike.  RCCL reads
 * NCCL_NCHANNELS_PER_PEER ONCE per process, so:
 *   - before the process's first communicator the library sets it to the
 *     count that communicator needs (nothing when that is 0, RCCL's default),
 *     unless the user set it, in which case the user's value holds for every
 *     communicator of the process and the rule is not applied;
 *   - a later communicator that needs a different count fails with
 *     GCMX_ERR_STATE (it would otherwise run silently with the first one's):
 *     pass the process's count explicitly (gcmx_comm_channels_per_peer of the
 *     first context), equal on every rank, or use a process of its own.
 * opt == NULL: global_x unknown, timeout from the environment, and
 * channels_per_peer / min_ctas / max_ctas from GCMX_COMM_CHANNELS_PER_PEER /
 * GCMX_COMM_MIN_CTAS / GCMX_COMM_MAX_CTAS when set (tuning), else automatic /
 * 16 / 32.  Without global_x the automatic rule of a multi-rank communicator
 * is RCCL's default (0). */
gcmx_status gcmx_comm_init_opts(gcmx_ctx* ctx, const uint8_t id[GCMX_UNIQUE_ID_BYTES],
                                int nranks, int rank, int left, int right,
                                const gcmx_comm_options* opt);
/* = gcmx_comm_init_opts(..., NULL). */
gcmx_status gcmx_comm_init(gcmx_ctx* ctx, const uint8_t id[GCMX_UNIQUE_ID_BYTES],
                           int nranks, int rank, int left, int right);
/* The channels per peer in effect for this context's communicator (0: RCCL's
 * default), -1 without one. */
int         gcmx_comm_channels_per_peer(const gcmx_ctx* ctx);
/* The automatic channels-per-peer rule as a pure function (no GPU call when
 * cus > 0): a one-rank communicator (nranks == 1) sizes it for its own slab of
 * local_x planes; a multi-rank one for the THINNEST slab of an even split,
 * floor(global_x / nranks) planes, whatever its own local_x (so ragged ranks
 * derive the same count), and 0 (RCCL's default) when global_x == 0.  The count
 * is from the CUs the one-pass step's interior launch of that slab (Y x Z
 * rows, borderSize bs, rows_per_block, 0 = automatic) leaves free on a device
 * of `cus` CUs (<= 0: the current device's): >= 16 -> 4, >= 8 -> 2, else 0
 * (DESIGN.md §5).  -1 for invalid arguments. */
int         gcmx_comm_channels_rule(int global_x, int nranks, int local_x, int Y, int Z, int bs,
                                    int rows_per_block, int cus);
/* ncclSend + ncclRecv calls this context's exchange groups posted so far (a
 * group that posts fewer than 2 x halo components x neighbours fails with
 * GCMX_ERR_COMM and aborts the communicator); -1 for a null context. */
long long   gcmx_comm_posted_calls(const gcmx_ctx* ctx);
/* Tests only: with on != 0 the context's exchange groups post their sends but
 * never their receives (a peer that never posts), so the exchange cannot
 * complete: the next bounded wait must return GCMX_ERR_COMM. */
gcmx_status gcmx_comm_test_stall(gcmx_ctx* ctx, int on);
/* Fill the X ghost layers of the current layer from the neighbours' boundary
 * inner planes (only the components the X stage reads), on the comm stream.
 * gcmx_step/gcmx_stage(axis 0) on a comm-enabled context call it themselves. */
gcmx_status gcmx_halo_exchange(gcmx_ctx* ctx);

/* In-process X slabs (one or several devices, one host thread): refresh the X
 * ghost layers of every slab's current layer from its neighbours in `slabs`
 * (ordered by increasing X; slabs[i] and slabs[i+1] must be adjacent).  Orders
 * itself after all pending work of every slab and before any later work of
 * any slab.  Call it before each time step, like the RCCL exchange. */
gcmx_status gcmx_halo_exchange_group(gcmx_ctx* const* slabs, int n);

/* In-process slab group: the RCCL X-slab exchange of gcmx_comm_init with
 * device-to-device copies (hipMemcpyPeerAsync on the contexts' comm streams)
 * instead of ncclSend/Recv, so the exchange code paths of gcmx_step (the
 * X-slab schedule: the new boundary planes posted while the interior runs,
 * the next step's boundary waiting for them) and of gcmx_stage(axis 0) run
 * unchanged on one or several devices of one process.  ctxs[i] becomes rank i
 * of n X-adjacent slabs (ordered by increasing X).  Like RCCL ranks, the
 * contexts must be driven concurrently, one host thread each (a wait for a
 * neighbour that never posts fails with GCMX_ERR_COMM after 60 s, or
 * GCMX_LOCAL_WAIT_SECONDS); the
 * semantics are those of the (dead) MPI slab design, src/test/TestMPI.cpp:33-50. */
gcmx_status gcmx_comm_init_local(gcmx_ctx* const* ctxs, int n);
/* Loopback transport, for timing ONE rank's step on one GPU: the context's X
 * slab exchanges with itself periodically (right inner planes -> left ghosts,
 * left inner -> right ghosts, the components the X stage reads) through the same
 * post / wait points as RCCL, by `blocks` 256-thread blocks of a copy kernel on
 * the comm stream that hold their CU slots for the time the bytes of one
 * direction take at `gbps_per_direction` (0: copy only) -- an xGMI transfer's
 * duration and CU footprint.  The physics is x-periodic (tests compare it with
 * gcmx_copy_box-filled periodic ghosts); bench only. */
gcmx_status gcmx_comm_init_loopback(gcmx_ctx* ctx, double gbps_per_direction, int blocks);
/* Drive an in-process group: one host thread per context, each calling
 * gcmx_step(ctxs[i], tau) `steps` times and then gcmx_sync.  The first failure
 * aborts the group and is returned (with its rank in gcmx_last_error). */
gcmx_status gcmx_local_group_steps(gcmx_ctx* const* ctxs, int n, double tau, int steps);

/* ---- simplex (tetrahedral) stage ----------------------------------------------
 * The device half of simplex::GridCharacteristicMethodInRiemannInvariants
 * (engine/simplex/GridCharacteristicMethodInRiemannInvariants.hpp:44-198) for one
 * body with the global calculation basis (BorderCalcMode::GLOBAL_BASIS,
 * SplittingType::PRODUCT, engine/simplex/Engine.cpp:117-148).  The mesh walk
 * (SimplexGrid::findCellCrossedByTheRay, SimplexGrid.cpp:57-164) is static for a
 * static mesh and basis, so the host resolves every characteristic foot once
 * (gcm_amd/host/simplex.cpp) and hands the result over as gsx_foot records.
 * Node arrays use the reference's per-vertex order (local vertex index), M = 9
 * doubles per node (AoS) at the boundary, SoA on the device. */
typedef struct gsx_ctx gsx_ctx;

typedef enum gsx_foot_kind {
	GSX_FOOT_CELL = 0,      /* foot inside a cell: hybridInterpolate (TetrahedronInterpolator.hpp:93-104) */
	GSX_FOOT_OUTER = 1,     /* outer invariant of a border node: 0 (:160-198, :57-95)  */
	GSX_FOOT_SPACETIME = 2, /* ray leaves through a border face: interpolateInSpaceTime
	                           (common.hpp:102-129) over the face's current and new values */
	GSX_FOOT_ZERO = 3       /* walk ended on a single vertex: u = 0 (:186-196, no branch) */
} gsx_foot_kind;

typedef struct gsx_foot {
	int kind;       /* gsx_foot_kind                                                 */
	int v[4];       /* CELL: the cell's vertices; SPACETIME: v[0..2] = the border face */
	int slot[4];    /* SPACETIME: value each weight multiplies, 0..2 = current layer of
	                   v[0..2], 3..5 = new layer of v[0..2] (interpolateInOwner order)  */
	double lam[4];  /* barycentric weights                                            */
	double q[3];    /* CELL: the foot (query point) for the gradient terms            */
} gsx_foot;

gcmx_status gsx_create(int device, int n_nodes, const double* coords /* [n][3] */, gsx_ctx** out);
void        gsx_destroy(gsx_ctx* ctx);
/* GcmMatrices of the inner basis: U, U1 [3 stages][9*9] row-major (ElasticModel<3>
 * ::constructGcmMatrices with the calculation basis, ElasticModel.hpp:57-65). */
gcmx_status gsx_set_matrices(gsx_ctx* ctx, const double* U, const double* U1);
/* Differentiation::estimateGradient (util/math/Differentiation.hpp:33-63): per node
 * its neighbours (CSR offsets[n+1], neighbors), the LSQ rows d (3 per entry), the
 * weights 1/|d|, the normal matrix A^T W A [9] and its determinant. */
gcmx_status gsx_set_gradient_plan(gsx_ctx* ctx, const int* offsets, const int* neighbors,
                                  const double* rows, const double* weights, const double* M,
                                  const double* det);
/* Feet of stage `stage`: feet[n_nodes][6] (invariants 0..5), the shift of each
 * invariant's characteristic (crossingPoints: direction * (-tau L(k)), [6][3]; a
 * CELL foot's q must equal coords + shift, the device recomputes it), the border
 * nodes (contactAndBorderStage) and the inner nodes (innerStage), in calculation order. */
gcmx_status gsx_set_stage_plan(gsx_ctx* ctx, int stage, const gsx_foot* feet, const double* shift,
                               int n_border, const int* border_nodes, int n_inner,
                               const int* inner_nodes);
gcmx_status gsx_upload(gsx_ctx* ctx, const double* aos /* [n][9] */);
gcmx_status gsx_download(gsx_ctx* ctx, double* aos);
/* Border correctors (engine/simplex/BorderCorrector.hpp:82-276, BorderCalcMode
 * GLOBAL_BASIS; replaces Engine::createMeshes' Border list, Engine.cpp:76-84, and
 * addBorderNode, :292-309).  Condition c has type[c] (gsx_border_type) and
 * min_det[c][s] = 1e-3 * getMaximalPossibleDeterminant at stage s
 * (BorderCorrector.hpp:131-133, 198-214).  Corrected node i is `nodes[i]` under
 * condition cond[i], with the border matrix B[i] (3 x 9, row-major,
 * ElasticModel::borderMatrixFixedForce / FixedVelocity of its normal,
 * ElasticModel.hpp:111-154), the local basis S[i] (3 x 3 row-major,
 * linal::createLocalBasis of the normal) and, per stage s, outer[s * n + i]:
 * the node's wave indices after contactAndBorderStage -- 0 none, 1 RIGHT
 * {1,3,5}, 2 LEFT {0,2,4}, 3 both (GridCharacteristicMethodInRiemannInvariants.hpp:71-88). */
typedef enum gsx_border_type { GSX_FIXED_FORCE = 0, GSX_FIXED_VELOCITY = 1 } gsx_border_type;
#define GSX_MAX_BORDER_CONDITIONS 16
gcmx_status gsx_set_border_plan(gsx_ctx* ctx, int n_cond, const int* type,
                                const double* min_det /* [n_cond][3] */, int n_nodes,
                                const int* nodes, const int* cond,
                                const double* B /* [n][27] */, const double* S /* [n][9] */,
                                const signed char* outer /* [3][n] */);
/* b(t) of every condition (BorderCondition::b, util/task/BorderCondition.hpp:33-40),
 * [n_cond][3]; used by the following gsx_plain_correction / gsx_stage calls. */
gcmx_status gsx_set_border_values(gsx_ctx* ctx, const double* b);
/* applyPlainCorrection on the current layer (BorderCorrector.hpp:177-187 ->
 * ElasticModel::applyPlainBorderCorrection, ElasticModel.hpp:202-228); the engine
 * calls it at construction and at the start of every step (Engine.cpp:44,99). */
gcmx_status gsx_plain_correction(gsx_ctx* ctx);
/* One stage: beforeStage (invariants + gradients), contactAndBorderStage,
 * the border correctors (applyInGlobalBasis, when a border plan is set),
 * innerStage, afterStage (U1) and the PRODUCT swap (engine/simplex/Engine.cpp:117-148).
 * gsx_stage = gsx_stage_nodes + gsx_stage_finish; a multi-body engine runs the
 * contact correctors (gsx_contact_correct) of every contact between the two halves
 * of every body, as Engine::gcmStage orders them (Engine.cpp:119-143). */
gcmx_status gsx_stage(gsx_ctx* ctx, int stage);
/* beforeStage + contactAndBorderStage (contact and border nodes' new invariants). */
gcmx_status gsx_stage_nodes(gsx_ctx* ctx, int stage);
/* border correctors + innerStage + afterStage + swap. */
gcmx_status gsx_stage_finish(gsx_ctx* ctx, int stage);
/* Thread layout of the node kernels (gradient, border, inner): 1 = one thread per
 * node (throughput layout for large meshes), 8 = eight lanes per node, one per
 * component / characteristic foot (latency layout for the reference's mesh
 * sizes: a node's dependent gathers run in parallel), 0 = automatic (8 below
 * 131 072 nodes).  Results are identical. */
gcmx_status gsx_set_node_lanes(gsx_ctx* ctx, int lanes);
/* gsx_stage in the eight-lane layout runs the border and inner halves of a stage
 * as ONE launch where the plan allows it (every inner foot that interpolates in
 * space-time with border nodes' new invariants waits, on the device, for exactly
 * those nodes): on = 1 (default) border + inner, 2 also the gradient groups in
 * the same launch, 0 separate launches, 3 (tuning only) mode 1 without the
 * 4096-block cap on the fused grid.  Results are identical.  In the one
 * launch a block takes its work index from an atomic ticket when it starts, so
 * it waits only on work that blocks already running took (no assumption on
 * dispatch order); every device-side wait is bounded and a timed-out wait is
 * reported by gsx_sync / gsx_download / the engine's run_steps.
 * gsx_last_stage_fused reports whether the last gsx_stage ran as one launch. */
gcmx_status gsx_set_stage_fusion(gsx_ctx* ctx, int on);
gcmx_status gsx_last_stage_fused(const gsx_ctx* ctx, int* fused);
/* Kernel launches made on the context's stream so far (each a dependent
 * kernel boundary of its step: the launch-floor model). */
gcmx_status gsx_launch_count(const gsx_ctx* ctx, long long* launches);
/* Tuning only: on = 3 is mode 1 without the 4096-block grid cap.  Every device
 * wait is bounded: a wait that gives up sets the context's error word, which
 * gsx_sync and gsx_download report (GCMX_ERR_STATE, "results invalid") and clear.
 * gsx_stage_plan_info: whether stage `stage`'s plan admits the one launch and
 * how many inner feet wait there for border nodes' new invariants.
 * gsx_set_wait_budget: polls per device wait (default 2^20); < 0 makes every
 * wait report a timeout at once (tests of the error path). */
gcmx_status gsx_stage_plan_info(const gsx_ctx* ctx, int stage, int* fusable, int* wait_feet);
gcmx_status gsx_set_wait_budget(gsx_ctx* ctx, int polls);

/* ---- simplex contact correctors ----------------------------------------------
 * ContactCorrectorInRiemannInvariants<Elastic, Elastic, AdhesionContactMatrixCreator>
 * (engine/simplex/ContactCorrector.hpp:303-419, 466-483) between two bodies on the
 * same device: one entry of Engine::contacts (Engine.hpp:36-47, Engine.cpp:220-287).
 * Pair i couples node nodes_a[i] of body a with nodes_b[i] of body b; normal[i]
 * is contactNormal of a towards b [n][3], S[i] = createLocalBasis(normal[i])
 * [n][9] row-major.  code_a / code_b [3][n]: per stage the node's wave indices
 * after matchInnersAndOuters (bits 0-1: 0 none, 1 RIGHT {1,3,5}, 2 LEFT {0,2,4},
 * 3 both; bit 2: the matching zeroed them).  min_det [3][2] = 1e-3 *
 * getMaximalPossibleDeterminants of each stage (ContactCorrector.hpp:250-276). */
typedef struct gsx_contact gsx_contact;
gcmx_status gsx_contact_create(gsx_ctx* a, gsx_ctx* b, int n, const int* nodes_a,
                               const int* nodes_b, const double* normal, const double* S,
                               const signed char* code_a, const signed char* code_b,
                               const double* min_det, gsx_contact** out);
void        gsx_contact_destroy(gsx_contact* c);
/* applyPlainCorrection (ContactCorrector.hpp:420-430 -> ElasticModel::
 * applyPlainContactCorrectionAsAverage, ElasticModel.hpp:239-272) on the current layers. */
gcmx_status gsx_contact_plain(gsx_contact* c);
/* applyInGlobalBasis at stage `stage` (ContactCorrector.hpp:333-348, 150-247) on the
 * new-layer invariants; call between gsx_stage_nodes and gsx_stage_finish of both bodies. */
gcmx_status gsx_contact_correct(gsx_contact* c, int stage);
/* One whole time step of a group of bodies and their contacts
 * (simplex::Engine::nextTimeStep after setBorderValues, engine/simplex/Engine.cpp:95-143:
 * plain corrections of the contacts then of the bodies, then for each stage every
 * body's gsx_stage_nodes, every contact's gsx_contact_correct, every body's
 * gsx_stage_finish) -- the same kernels as those calls, captured once per layer
 * state into a HIP graph and replayed, so a step costs one launch instead of
 * ~12 (the reference's mesh sizes are launch-bound).  Border values are read
 * from device memory written by gsx_set_border_values, so they may change
 * every step.  Results are identical to the individual calls. */
gcmx_status gsx_step(gsx_ctx* const* bodies, int n_bodies, gsx_contact* const* contacts,
                     int n_contacts);
gcmx_status gsx_sync(gsx_ctx* ctx);
/* Tests only: the device interpolation the simplex stage kernels run, on given
 * inputs.  Case i: v[4i..], g[(4i+j)*3..] (vertex j's gradient), c[(4i+j)*3..]
 * (vertex j), q[3i..], lam[4i..] (q's barycentrics, as the host plan computes
 * them); out[2i] = TetrahedronInterpolator::hybridInterpolate
 * (TetrahedronInterpolator.hpp:93-104, a CELL foot), out[2i+1] = the linear
 * form lam . v (hpp:27-37; interpolateInOwner's value, a SPACETIME foot). */
gcmx_status gsx_test_interpolate(int device, int n, const double* v, const double* g, const double* c,
                                 const double* q, const double* lam, double* out);

/* ---- synchronisation and timing ------------------------------------------- */
gcmx_status gcmx_sync(gcmx_ctx* ctx);
/* The context's compute stream as a hipStream_t (for event timing by callers). */
void*       gcmx_stream(gcmx_ctx* ctx);
/* Per-kernel event timing on the stream each kernel is launched on: when
 * enabled, every launch is bracketed by hipEvents and its duration added to
 * the kernel's bucket once the events complete (read after gcmx_sync). */
gcmx_status gcmx_profile_enable(gcmx_ctx* ctx, int enable);
gcmx_status gcmx_profile_reset(gcmx_ctx* ctx);
/* Returns the number of kernel buckets; fills name/total_ms/launches of
 * bucket `index` when index < count. */
int         gcmx_profile_read(gcmx_ctx* ctx, int index, const char** name,
                              double* total_ms, long long* launches,
                              double* bytes_per_launch);
/* The kernel instance the last launch of bucket `index` ran (e.g.
 * "k_step_tx2<2, 512, KF0, UNI, !FACES>"); "" when unknown. */
const char* gcmx_profile_kernel(gcmx_ctx* ctx, int index);

/* Device-side layout facts (for DESIGN.md-style reporting and tests). */
long long   gcmx_inner_nodes(gcmx_ctx* ctx);
long long   gcmx_all_nodes(gcmx_ctx* ctx);
size_t      gcmx_device_bytes(gcmx_ctx* ctx);
/* Measurement only (bench.py's roofline.copy_ceiling): the practical HBM rate
 * of this device for a flat copy of `bytes` bytes (half read, half written;
 * 16 B per lane, non-temporal stores, 32 768 blocks of 256 threads, grid-stride:
 * the fastest of the flat-copy shapes tools/copy_probe.hip times).  Median of `reps` timed copies
 * after one warm copy; *ms_out = that copy's duration (HIP events on the
 * ctx stream).  Allocates and frees 2 x bytes / 2 on the context's device. */
gcmx_status gcmx_copy_ceiling(gcmx_ctx* ctx, size_t bytes, int reps, float* ms_out);
/* Measurement only: out[0], out[1] = device addresses of the two time layers as
 * allocated (layer A holds the state after an even number of steps), out[2] =
 * bytes per layer, out[3] = how they are allocated: both live in one block
 * (the default: layer A, a 2 MiB gap, layer B; environment GCMX_LAYER_GAP =
 * bytes of the gap at gcmx_create, < 0 = two separate allocations: out[3] = 0)
 * which is, by default once it spans two chunks (256 MiB from an 8 GiB block
 * up, else 64 MiB), physical chunks mapped in a shuffled order (out[3] = the
 * chunk bytes); GCMX_ALLOC=malloc gives one
 * hipMalloc (1), =contiguous a physically contiguous block (2), =shuffle:<MiB>
 * another chunk size.  DESIGN.md §2 has the measurements. */
gcmx_status gcmx_layer_info(gcmx_ctx* ctx, uint64_t out[4]);
/* The device layout of a layer (tests, tools): out[0..2] = the element strides
 * of axes 0..2 (x plane, y row, z), out[3] = elements per component plane,
 * out[4] = the element offset of inner node (0, 0, 0) in a plane, out[5] = the
 * padded row length.  Host code never needs it (gcmx_upload / gcmx_download
 * take the reference's all-nodes AoS order); GCMX_ROW_PAD / GCMX_PLANE_PAD /
 * GCMX_CS_PAD (elements, read at gcmx_create, tests only) pad rows, 3-D x
 * planes and component planes so a test can check that nothing derives a
 * stride from the sizes. */
gcmx_status gcmx_geometry(gcmx_ctx* ctx, int64_t out[6]);
/* Measurement only: the shader clock under load.  _start launches ONE wave on
 * a stream of its own that records (s_memrealtime, s_memtime) pairs every
 * `period_us` for `seconds` (it co-resides with the kernels that run meanwhile);
 * _read waits for it and copies up to `cap` pairs into samples[2*i], [2*i+1]
 * (100 MHz ticks, shader cycles); returns the number taken, -1 on error.
 * Clock over an interval = Δcycles / Δticks × 100 MHz. */
gcmx_status gcmx_clock_probe_start(gcmx_ctx* ctx, double seconds, double period_us);
int         gcmx_clock_probe_read(gcmx_ctx* ctx, uint64_t* samples, int cap);

#ifdef __cplusplus
}
#endif
#endif /* GCMX_H */
