// simplex.hpp -- host side of the simplex (tetrahedral) grid-characteristic path.
//
// The reference's simplex engine (engine/simplex/*, grid/simplex/*) runs the
// grid-characteristic method in Riemann invariants
// (GridCharacteristicMethodInRiemannInvariants.hpp:44-198) on a CGAL
// triangulation.  CGAL is not in this image, so the mesh here is built by
// boxMesh() (a jittered Kuhn tetrahedralisation of a box) and the triangulation
// queries the method needs -- incident cells, face neighbours, the line walk
// of LineWalker.hpp / SimplexGrid.cpp:57-164 -- are restated over it.
//
// The mesh is static and the calculation basis constant, so everything the
// walk decides (the cell or border face each characteristic foot falls in,
// barycentric weights, which invariants are outer at a border node) is found
// once on the host (StagePlan).  The per-step work -- Riemann invariants, LSQ
// gradients (Differentiation.hpp:33-63), hybrid interpolation
// (TetrahedronInterpolator.hpp:93-104), space-time interpolation
// (common.hpp:102-129), U1 back-transform -- runs on the GPU (gsx_* in
// include/gcmx.h, gcm_amd/csrc/simplex.hip).
#pragma once

#include <array>
#include <chrono>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gcmx.h"
#include "elastic_model.hpp"
#include "task.hpp"

namespace gcm {
namespace simplex {

constexpr real EQUALITY_TOLERANCE = 1e-9;           // util/infrastructure/Types.hpp:10
constexpr int MAX_NUMBER_OF_NEIGHBOR_VERTICES = 20;  // Cgal3DTriangulation.hpp:53

/// Grid::EmptySpaceFlag (SimplexGrid.hpp): the grid id of cells outside every body.
constexpr int EMPTY_SPACE = -1;

/// Tetrahedral mesh of one body: vertex coordinates, positively oriented cells,
/// face neighbours (nb[c][i] = cell across the face opposite vertex i, -1 =
/// outside the body) and vertex -> incident cells (ascending cell index).
/// A body cut out of a Triangulation also knows, for every face with nb < 0,
/// the grid id on the other side (nbGrid: EMPTY_SPACE or another body) and, for
/// every vertex, the other grid ids of the cells around it (otherGrids, sorted,
/// EMPTY_SPACE for the box surface) -- SimplexGrid::gridsAroundVertex
/// (SimplexGrid.hpp:415-423) minus the body's own id.
struct TetMesh {
	std::vector<Real3> v;
	std::vector<std::array<int, 4>> cells;
	std::vector<std::array<int, 4>> nb;
	std::vector<int> incOff, incCells;
	std::vector<std::array<int, 4>> nbGrid;
	std::vector<std::vector<int>> otherGrids;
	std::vector<int> global;  // local vertex -> vertex of the triangulation
	void buildTopology();
	int nVertices() const { return (int)v.size(); }
};

/// The global triangulation of the calculation space (the CgalTriangulation
/// every SimplexGrid of the task shares, SimplexGrid.cpp:12-37): the box mesh and
/// a grid id per cell (EMPTY_SPACE outside the domain surface).
struct Triangulation {
	TetMesh all;
	std::vector<int> gridId;
};

/// Odd-parity inside test of a closed triangulated surface (the .off domain):
/// the generalized winding number rounded to an integer, inside when odd.
bool offContains(const std::vector<Real3>& points, const std::vector<std::array<int, 3>>& faces,
                 const Real3& p);

/// InmMeshLoader::readFromFile (grid/simplex/mesh_loaders/InmMeshLoader.hpp:96-170):
/// points, cells (1-based INM vertex numbers) and the material of every cell.
void readInm(const std::string& fileName, std::vector<Real3>& points,
             std::vector<std::array<int, 4>>& cells, std::vector<int>& materials);

/// Read the vertices and triangles of an .off file (the reference meshes/*.off).
void readOff(const std::string& fileName, std::vector<Real3>& points,
             std::vector<std::array<int, 3>>& faces);

/// Kuhn tetrahedralisation (6 tetrahedra per cube) of the box [lo, hi] with
/// n cubes per axis.  Vertices are jittered by up to `jitter` * h with a
/// SplitMix64 stream of `seed`: interior vertices in 3-D, face vertices within
/// their face, edge vertices along their edge, corners fixed.
TetMesh boxMesh(const std::array<int, 3>& n, const Real3& lo, const Real3& hi, real jitter,
                uint64_t seed);

/// The task's triangulation: boxMesh of Task::SimplexGrid, cells outside the
/// .off domain marked EMPTY_SPACE, the others assigned to bodies by bodyAreas.
Triangulation buildTriangulation(const Task& task);

/// The cells of body `id` with their vertices renumbered in ascending global
/// order (SimplexGrid's constructor collects vertexHandles into a std::set,
/// SimplexGrid.cpp:18-30), neighbour grid ids and vertex states.
TetMesh bodyMesh(const Triangulation& tr, int id);

/// SimplexGrid<3> (grid/simplex/SimplexGrid.{hpp,cpp}) over the TetMesh of one body.
class Grid {
public:
	explicit Grid(const TetMesh& mesh);
	const TetMesh& mesh;
	/// Cell found by the ray walk: n = 4 (cell), 3 (border face), 2, 1, 0.
	struct Cell {
		int n = 0;
		int v[4] = {-1, -1, -1, -1};
	};
	bool isInner(int it) const { return inner[it]; }
	/// SimplexGrid::normal (SimplexGrid.hpp:426-444) over the faces whose outer
	/// grid id satisfies `use`: borderNormal (EMPTY_SPACE, :151-154),
	/// contactNormal (one neighbour grid, :141-144), commonNormal (any, :157-160).
	template <typename Pred> Real3 normal(int it, Pred use) const;
	Real3 borderNormal(int it) const;
	Real3 contactNormal(int it, int other) const;
	Real3 commonNormal(int it) const;
	/// findNeighborVertices (SimplexGrid.hpp:249-259): ascending local indices
	std::vector<int> neighborVertices(int it) const;
	/// findCellCrossedByTheRay (SimplexGrid.cpp:57-112)
	Cell findCellCrossedByTheRay(int it, const Real3& shift) const;
	real averageHeight = 0, minimalHeight = 0;  // collectCellHeightsStatistics (Histogram)
	/// markInnersAndBorders (SimplexGrid.cpp:216-252): contact, border (with
	/// multicontact) and inner nodes, each in ascending local order
	std::vector<int> innerIdx, borderIdx, contactIdx;

private:
	std::vector<char> inner;
	const Real3& P(int vtx) const { return mesh.v[vtx]; }
	int otherVertexIndex(int cell, int a, int b, int c) const;
	int findCrossedIncidentCell(int vh, const Real3& query, real eps) const;
	void findCrossedInsideOutFacet(int t, const Real3& q, const Real3& p, int& a, int& b, int& c,
	                               real eps) const;
	std::vector<int> collectCells(const Real3& q, const Real3& p, int t, int u, int v, int w,
	                              std::array<int, 3>& lastFace) const;
	std::vector<int> cellsAlongSegmentFromVertex(int q, const Real3& p,
	                                             std::array<int, 3>& lastFace) const;
	std::vector<int> cellsAlongSegmentFromCell(int t, const Real3& q, const Real3& p,
	                                           std::array<int, 3>& lastFace) const;
	Cell checkLineWalkFoundCell(int it, const std::vector<int>& cells,
	                            const std::array<int, 3>& lastFace, const Real3& start,
	                            const Real3& query) const;
};

/// Static data of one stage for the device (gsx_set_stage_plan).
struct StagePlan {
	std::vector<gsx_foot> feet;  // [node][6] invariants 0..5 (6..8 have dx == 0)
	double shift[6][3] = {};     // direction * dx(k) (crossingPoints, common.hpp:46-52)
	std::vector<int> borderNodes, innerNodes;
	/// waveIndices of every node after contactAndBorderStage: 0 none, 1 RIGHT,
	/// 2 LEFT, 3 both (gsx_set_border_plan's outer codes)
	std::vector<signed char> outerCode;
};

/// Border correctors of the body: the Border list of Engine::createMeshes
/// (engine/simplex/Engine.cpp:76-84) filled by addBorderNode (:292-309), with
/// the per-node data BorderCorrectorInPdeVectors needs (gsx_set_border_plan).
struct BorderPlan {
	std::vector<int> type;           // per condition (gsx_border_type)
	std::vector<double> minDet;      // [cond][3]
	std::vector<int> nodes, cond;    // corrected nodes and their condition
	std::vector<double> normal;      // [n][3] commonNormal
	std::vector<double> B, S;        // [n][27] border matrix, [n][9] local basis
	std::vector<signed char> outer;  // [3][n]
};

/// The LSQ gradient operator of every node (gsx_set_gradient_plan).
struct GradientPlan {
	std::vector<int> offsets, neighbors;
	std::vector<double> rows, weights, M, det;
};

/// Differentiation::estimateGradient's per-node matrices (Differentiation.hpp:33-63).
GradientPlan buildGradientPlan(const Grid& grid);

/// Feet of every node for stage s along `direction` with crossing points
/// dx = -tau * L (common.hpp:46-52) -- GridCharacteristicMethodInRiemannInvariants
/// ::interpolateValuesAround (:156-198) decided once, plus the outer-invariant
/// bookkeeping of contactAndBorderStage (:57-95).
StagePlan buildStagePlan(const Grid& grid, const Real3& direction, const real L[9], real tau);

/// linal::barycentricCoordinates of a tetrahedron (linal/geometry.hpp:142-151).
std::array<real, 4> barycentricCoordinates(const Real3& a, const Real3& b, const Real3& c, const Real3& d,
                                           const Real3& q);
/// TetrahedronInterpolator::interpolateInOwner's choice (util/math/interpolation/
/// TetrahedronInterpolator.hpp:113-155): the tetrahedron of the six points that
/// holds q (its point indices) and q's barycentrics in it; throws when none does.
/// The stage plan's space-time feet use it; the interpolated value is then
/// lam[0] v[slot[0]] + ... + lam[3] v[slot[3]] (on the device).
void interpolateInOwnerPick(const Real3 (&pts)[6], const Real3& q, int (&slot)[4], real (&lam)[4]);

/// ElasticModel::borderMatrixFixedForce / borderMatrixFixedVelocity
/// (rheology/models/ElasticModel.hpp:111-154), 3 x 9 row-major.
std::array<real, 27> borderMatrix(BorderConditions::T type, const Real3& normal);

BorderPlan buildBorderPlan(const Task& task, const Grid& grid, const GcmMatrices<3>& matrices,
                           const real calc[3][3], const StagePlan stages[3]);

}  // namespace simplex
}  // namespace gcm

#include "engine.hpp"
#include "snapshot.hpp"

namespace gcm {
namespace simplex {

/// One contact of Engine::contacts (engine/simplex/Engine.hpp:36-47): the node
/// pairs addContactNode collected (Engine.cpp:273-287) in triangulation order,
/// with the static data ContactCorrectorInRiemannInvariants needs per stage.
struct ContactPlan {
	size_t a = 0, b = 0;               // indices into HostPlans::bodies (ids a < b)
	ContactConditions::T condition = ContactConditions::T::ADHESION;
	std::vector<int> nodesA, nodesB;   // local vertex indices
	std::vector<double> normal;        // [n][3] contactNormal of A towards B
	std::vector<double> S;             // [n][9] createLocalBasis(normal), row-major
	/// [3][n] per side: wave indices after matchInnersAndOuters
	/// (ContactCorrector.hpp:365-397): bits 0-1 = 0 none, 1 RIGHT, 2 LEFT, 3 both;
	/// bit 2 = the matching zeroed those invariants (odd N)
	std::vector<signed char> codeA, codeB;
	double minDet[3][2] = {};          // 1e-3 * getMaximalPossibleDeterminants (:250-276)
};

/// Everything simplex::Engine's constructor builds for one body.
struct BodyPlans {
	size_t id = 0;
	TetMesh mesh;
	real averageHeight = 0, maximalEigenvalue = 0;
	GcmMatrices<3> matrices;
	GradientPlan gradient;
	StagePlan stages[3];
	BorderPlan border;
	std::vector<real> pde;  // initial layer, 9 per vertex
	std::vector<int> borderIdx, innerIdx, contactIdx;
};

/// GPU-free set-up of the simplex path: the task's bodies (ascending ids), their
/// contacts (Utils::makePairs order) and the time step.
struct HostPlans {
	real tau = 0;
	std::vector<BodyPlans> bodies;
	std::vector<ContactPlan> contacts;
};
HostPlans buildHostPlans(const Task& task);

/// simplex::Engine<3, CgalTriangulation> (engine/simplex/Engine.{hpp,cpp}) for
/// isotropic-elastic bodies: GcmType ADVECT_RIEMANN_INVARIANTS, SplittingType
/// PRODUCT, BorderCalcMode GLOBAL_BASIS, constant Task::calculationBasis,
/// Task::borderConditions through the border correctors (FIXED_FORCE,
/// FIXED_VELOCITY) and ADHESION contacts through the contact correctors; border
/// nodes no condition covers keep zero outer invariants.
class Engine : public AbstractEngine {
public:
	explicit Engine(const Task& task, int device = 0);
	~Engine() override;
	size_t numberOfBodies() const { return bodies.size(); }
	const TetMesh& mesh(size_t body = 0) const { return bodies.at(body).mesh; }
	/// current layer of a body, 9 doubles per vertex (downloads)
	std::vector<real> pde(size_t body = 0) const;
	real timeStepValue() const { return tau; }
	/// wait for every body's stream (timing)
	void sync() const;
	size_t numberOfContactPairs() const;
	/// Run each step as one replayed HIP graph (gsx_step) or as the individual
	/// stage calls (default); identical results.  Measured equal speed on MI355X:
	/// the step is bound by the kernels' own duration, not by launches.
	void setReplaySteps(bool on) { replaySteps = on; }
	/// Thread layout of every body's node kernels (gsx_set_node_lanes: 0 auto, 1, 8).
	void setNodeLanes(int lanes);
	/// One launch per stage for the border and inner halves of a body without
	/// contacts (gsx_set_stage_fusion: 0 off, 1 border + inner, 2 with the
	/// gradient; -1, the default: measured per mesh -- the engine's first steps
	/// run kTuneSteps in mode 1 and kTuneSteps in mode 2 between stream
	/// synchronisations and keep mode 2 only where it is >= 3 % faster; the
	/// modes give identical results, so the measured steps are ordinary steps).
	void setStageFusion(int mode);
	/// the mode in effect (1 or 2 while / after measuring in mode -1), and
	/// whether the automatic choice is still being measured
	int stageFusion() const { return fusionMode_; }
	bool fusionTuning() const { return autoFusion_ && tunePhase_ < 3; }
	/// measured ms per step of modes 1 and 2 (automatic mode; 0 before)
	std::pair<double, double> fusionTimes() const { return {tuneMs_[0], tuneMs_[1]}; }
	/// kernel launches made on the bodies' streams since construction
	/// (gsx_launch_count): the dependent launches of the steps
	long long launches() const;
	static constexpr int kTuneSteps = 8;
	/// stages run as one launch since construction
	long long fusedStages() const { return fusedStages_; }
	/// (plan admits the one launch, inner feet that wait there) of a body's stage
	std::pair<bool, int> stagePlanInfo(size_t body, int stage) const;
	/// polls per device wait of the one-launch stages (gsx_set_wait_budget; < 0:
	/// every wait reports a timeout, for tests of the error path)
	void setWaitBudget(int polls);

protected:
	void nextTimeStep() override;
	real estimateTimeStep() override;
	void writeSnapshots(const int step) override;

private:
	bool autoFusion_ = true;  // stage fusion mode measured per mesh (setStageFusion(-1))
	int fusionMode_ = 1;
	int tunePhase_ = 0;       // 0: warm-up step, 1 / 2: timing mode 1 / 2, 3: chosen
	int tuneLeft_ = 0;
	double tuneMs_[2] = {0.0, 0.0};
	std::chrono::steady_clock::time_point tuneT0_;
	void stepCalls();

	struct Body {
		size_t id = 0;
		int materialNumber = 0;
		TetMesh mesh;
		gsx_ctx* ctx = nullptr;
		bool hasBorderPlan = false;
	};
	std::vector<Body> bodies;
	std::vector<gsx_contact*> contacts;
	size_t contactPairs = 0;
	real tau = 0;
	std::vector<Task::BorderCondition> conditions;
	std::unique_ptr<VtkSnapshotter> vtk;
	int stepsPerSnap = 1;
	bool replaySteps = false;
	long long fusedStages_ = 0;
	void setBorderValues(real time);
	void plainCorrections();
};

}  // namespace simplex
}  // namespace gcm
