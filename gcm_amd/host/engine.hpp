// engine.hpp -- host mirror of libgcm's cubic engine surface over the gcmx C-ABI.
//
// Same class roles and call order as the reference:
//   AbstractEngine (engine/AbstractEngine.{hpp,cpp})        -> gcm::AbstractEngine
//   Clock (engine/GlobalVariables.hpp:16-41)                 -> gcm::Clock
//   cubic::Engine<D> (engine/cubic/Engine.{hpp,cpp})         -> gcm::cubic::Engine<D>
//   cubic::AbstractFactoryBase / AbstractFactory             -> cubic::AbstractFactoryBase / HipFactory
//   cubic::AbstractMesh / DefaultMesh                        -> cubic::AbstractMesh / HipMesh
//   cubic::GridCharacteristicMethodBase / ...Method<Mesh>    -> same base / HipGridCharacteristicMethod
//   cubic::AbstractBorderConditions / BorderConditions       -> same base / HipBorderConditions
//   cubic::AbstractContactCopier / ContactCopier             -> same base / HipContactCopier
// The per-node work of stage(), border fills and contact copies runs on the GPU
// through include/gcmx.h; the host keeps set-up and the time loop.
#pragma once

#include <map>
#include <memory>
#include <vector>

#include "../../include/gcmx.h"
#include "snapshot.hpp"
#include "task.hpp"

namespace gcm {

/// engine/GlobalVariables.hpp:16-41 -- physical time and time step.
struct Clock {
	static real Time() { return time; }
	static real TimeStep() { return timeStep; }

private:
	static real time;
	static real timeStep;
	static void setZero() { time = timeStep = 0; }
	static void tickTack() { time += timeStep; }
	friend class AbstractEngine;
};

/// Throw gcm::Exception for a failed gcmx call.
void gcmxCheck(gcmx_status s, const char* what);

/// engine/AbstractEngine.hpp:29-55
class AbstractEngine {
public:
	explicit AbstractEngine(const Task& task);
	virtual ~AbstractEngine() = default;
	AbstractEngine(const AbstractEngine&) = delete;
	AbstractEngine& operator=(const AbstractEngine&) = delete;
	/// AbstractEngine::run (AbstractEngine.cpp:30-46)
	void run();
	/// `n` more time steps of the same loop body, ignoring requiredTime (benchmarks).
	void runSteps(int n);
	int stepsDone() const { return steps; }
	real getRequiredTime() const { return requiredTime; }

protected:
	const real CourantNumber = 0;
	real requiredTime = 0;
	int steps = 0;
	void afterConstruction(const Task& task);
	virtual void nextTimeStep() = 0;
	virtual real estimateTimeStep() = 0;
	virtual void writeSnapshots(const int step) = 0;
};

/// grid/AbstractGrid.hpp -- what stage()/apply() receive and downcast.
class AbstractGrid {
public:
	virtual ~AbstractGrid() = default;
};

namespace cubic {

/// CubicGrid<D> (grid/cubic/CubicGrid.hpp) -- index arithmetic of the reference
/// storage order (X slowest); `it` are local indices, ghosts at -bs..-1 / size..
template <int D>
struct CubicGrid : public AbstractGrid {
	typedef std::array<int, D> IntD;
	typedef std::array<real, D> RealD;
	struct ConstructionPack {
		int borderSize = 0;
		IntD sizes{};
		IntD start{};
		RealD h{};
	};
	CubicGrid(size_t id_, const ConstructionPack& cp);
	size_t id;
	int borderSize;
	IntD sizes, start;
	RealD h;
	long long indexMaker[D];
	long long sizeOfAllNodes() const { return indexMaker[0] * (2LL * borderSize + sizes[0]); }
	long long getIndex(const IntD& it) const {
		long long a = 0;
		for (int i = 0; i < D; i++) a += indexMaker[i] * (long long)(it[i] + borderSize);
		return a;
	}
	/// coords (CubicGrid.hpp:114-126): startR + it * h, padded to 3-D
	Real3 coords(const IntD& it) const {
		Real3 c = {0, 0, 0};
		for (int i = 0; i < D; i++) c[i] = (real)start[i] * h[i] + (real)it[i] * h[i];
		return c;
	}
	real getMinimalSpatialStep() const;
	/// AABB in global indices {start, start + sizes - 1}
	std::pair<IntD, IntD> aabb() const;
};

/// engine/cubic/AbstractMesh.hpp:17-51
template <int D>
class AbstractMesh : public CubicGrid<D> {
public:
	using CubicGrid<D>::CubicGrid;
	virtual ~AbstractMesh() = default;
	virtual void setUpPde(const Task& task) = 0;
	virtual real getMaximalEigenvalue() const = 0;
	virtual void swapCurrAndNextPdeTimeLayer(int indexOfNextPde) = 0;
};

/// Host half of DefaultMesh::setUpPde (DefaultMesh.hpp:60-66): the PDE layer
/// after MaterialsCondition::apply + InitialCondition::apply in the reference
/// AoS all-nodes order, the material-condition index of every node (0 =
/// default, i = i-th area condition) and the GcmMatrices per condition.
/// No GPU involved; HipMesh::setUpPde uploads it.
template <int D>
struct HostState {
	std::vector<real> pde;
	std::vector<uint8_t> matId;
	std::vector<GcmMatrices<D>> matrices;
	std::vector<real> tau0;  // IsotropicMaterial::tau0 per material condition
	std::vector<int> materialNumber;  // IsotropicMaterial::materialNumber per condition
	real maximalEigenvalue = 0;
};

/// Engine::createGridsAndContacts's ConstructionPack for body `id` (Engine.cpp:38-60).
template <int D>
typename CubicGrid<D>::ConstructionPack constructionPack(const Task& task, size_t id);

template <int D>
HostState<D> buildHostState(const Task& task, const CubicGrid<D>& grid);

/// DefaultMesh's role with GPU-resident storage: the context owns both time
/// layers on the device; the host holds only set-up data.
template <int D>
class HipMesh : public AbstractMesh<D> {
public:
	static constexpr int M = pdeSize(D);
	typedef typename CubicGrid<D>::IntD IntD;
	HipMesh(const Task& task, size_t id, const typename CubicGrid<D>::ConstructionPack& cp,
	        int device);
	~HipMesh() override;
	/// DefaultMesh::setUpPde (DefaultMesh.hpp:60-66): allocate, MaterialsCondition,
	/// InitialCondition, then upload.
	void setUpPde(const Task& task) override;
	real getMaximalEigenvalue() const override { return maximalEigenvalue; }
	/// The device swap happens inside gcmx_stage; nothing to do here.
	void swapCurrAndNextPdeTimeLayer(int) override {}
	gcmx_ctx* ctx() const { return ctx_; }
	/// Current layer in the reference AoS all-nodes order (downloads).
	std::vector<real> pdeAll() const;
	/// One node's PDE vector (downloads the layer; for tests and snapshots).
	std::array<real, M> pde(const IntD& it) const;
	int numberOfMaterials() const { return (int)matrices.size(); }
	/// tau0 of the materials in the device table order (gcmx_set_materials).
	const std::vector<real>& deviceTau0() const { return deviceTau0_; }
	/// Material-condition index per node (all-nodes order) and the conditions'
	/// IsotropicMaterial::materialNumber (DefaultMesh::material(it), for snapshots).
	const std::vector<uint8_t>& materialIdsAll() const { return matIdAll_; }
	const std::vector<int>& materialNumbers() const { return materialNumbers_; }

	/// STACKS.  3-D bodies stacked along y or z whose every contact is an adhesion
	/// contact over a whole face (equal sizes and starts on the other two axes)
	/// run as ONE grid, the stack: ContactCopier::apply fills a body's ghost layers
	/// at the contact with the neighbour's current layer right before the stage of
	/// the contact's axis (Engine.cpp:99-107, ContactConditions.hpp:56-68) -- what
	/// the stack's stage reads there anyway -- so every inner node is bitwise that
	/// of the separate bodies (TestEngine.cpp:27-87 pins split == unsplit), and the
	/// step keeps the one-pass kernel instead of three per-stage passes.  A member
	/// keeps its own host data (set-up, materials, snapshots) and reads its part of
	/// the stack's device layers; the stack is a HipMesh over the combined box.
	void joinStack(const std::shared_ptr<HipMesh<D>>& stack, int axis, int offset);
	const std::shared_ptr<HipMesh<D>>& stackMesh() const { return stack_; }
	/// A stack member's DefaultMesh::setUpPde, host half only (the stack uploads).
	HostState<D> setUpMember(const Task& task);
	/// The stack's set-up from its members' host states, members in stack order.
	void setUpStack(const std::vector<std::shared_ptr<HipMesh<D>>>& members,
	                const std::vector<HostState<D>>& states);

private:
	std::shared_ptr<HipMesh<D>> stack_;  // set for a stack member
	int stackAxis_ = -1, stackOffset_ = 0;
	bool ownsCtx_ = true;
	gcmx_ctx* ctx_ = nullptr;
	int device;
	real maximalEigenvalue = 0;
	std::vector<GcmMatrices<D>> matrices;  // one per material condition
	std::vector<real> deviceTau0_;
	std::vector<uint8_t> matIdAll_;
	std::vector<int> materialNumbers_;
	bool pdeIsSetUp = false;
};

/// engine/cubic/GridCharacteristicMethod.hpp:13-17
class GridCharacteristicMethodBase {
public:
	virtual ~GridCharacteristicMethodBase() = default;
	virtual void stage(const int s, const real& timeStep, AbstractGrid& mesh) const = 0;
};

/// GridCharacteristicMethod<Mesh>::stage on the device (gcmx_stage).
template <int D>
class HipGridCharacteristicMethod : public GridCharacteristicMethodBase {
public:
	explicit HipGridCharacteristicMethod(const Task&) {}
	void stage(const int s, const real& timeStep, AbstractGrid& mesh) const override;
	/// All D stages at once (gcmx_step; fused kernels where admissible).
	void step(const real& timeStep, HipMesh<D>& mesh) const;
};

/// engine/cubic/BorderConditions.hpp:17-20
class AbstractBorderConditions {
public:
	virtual ~AbstractBorderConditions() = default;
	virtual void apply(AbstractGrid& mesh, const int direction) const = 0;
	virtual bool empty() const = 0;
	/// Every face uniform: each node of a face has the same last-applying
	/// condition, or none has any (then gcmx_step_faces runs the whole step).
	virtual bool uniformFaces() const { return false; }
	/// gcmx_face per face (2*D entries, faces[2*axis + side]) at Clock::Time().
	virtual void faces(gcmx_face*) const {}
	/// Non-uniform faces held as a per-node face map (gcmx_face_map): the whole
	/// step runs through gcmx_step_face_map.  Null when there is none.
	virtual const gcmx_face_map* faceMap() const { return nullptr; }
	/// Every condition's quantities at Clock::Time() (the face map's conditions).
	virtual int conditionsAt(gcmx_face*) const { return 0; }
};

/// BorderConditions<Mesh> (BorderConditions.hpp:23-121): node lists found on the
/// host at construction (:46-78) and uploaded to the device once; ghost fills
/// on the device per stage (:81-114), enqueued without host synchronisation.
/// When every face is uniform the engine runs whole steps (gcmx_step_faces).
template <int D>
class HipBorderConditions : public AbstractBorderConditions {
public:
	HipBorderConditions(const Task& task, const HipMesh<D>& mesh);
	~HipBorderConditions() override;
	HipBorderConditions(const HipBorderConditions&) = delete;
	HipBorderConditions& operator=(const HipBorderConditions&) = delete;
	void apply(AbstractGrid& mesh, const int direction) const override;
	bool empty() const override { return conditions.empty(); }
	bool uniformFaces() const override { return uniform; }
	void faces(gcmx_face* out) const override;
	const gcmx_face_map* faceMap() const override { return faceMap_; }
	int conditionsAt(gcmx_face* out) const override;

private:
	struct Condition {
		int direction;
		std::vector<int> leftNodes, rightNodes;  // D ints per node
		gcmx_border_nodes* leftD = nullptr;      // the same lists on the device
		gcmx_border_nodes* rightD = nullptr;
		std::vector<std::pair<PhysicalQuantities::T, Task::TimeDependency>> values;
	};
	std::vector<Condition> conditions;
	bool uniform = false;
	std::array<int, 6> faceCondition{{-1, -1, -1, -1, -1, -1}};  // per face: condition or -1
	gcmx_face_map* faceMap_ = nullptr;  // non-uniform faces, <= GCMX_MAX_FACE_CONDITIONS conditions
};

/// engine/cubic/ContactConditions.hpp:20-68 (adhesion: plain copy)
template <int D>
class HipContactCopier {
public:
	HipContactCopier(const std::array<int, 3>& dstMin, const std::array<int, 3>& dstMax,
	                 const std::array<int, 3>& srcMin)
	    : dmin(dstMin), dmax(dstMax), smin(srcMin) {}
	void apply(HipMesh<D>& a, const HipMesh<D>& b) const;

private:
	std::array<int, 3> dmin, dmax, smin;
};

/// rheology/ode/Ode.hpp:16-19
class AbstractOde {
public:
	virtual ~AbstractOde() = default;
	virtual void apply(AbstractGrid& mesh, const real timeStep) = 0;
};

/// MaxwellViscosityOde<Mesh> (rheology/ode/Ode.hpp:24-38) on the device:
/// sigma *= exp(-timeStep / tau0) per node (gcmx_ode_maxwell).
template <int D>
class HipMaxwellViscosityOde : public AbstractOde {
public:
	void apply(AbstractGrid& mesh, const real timeStep) override;
};

/// VtkSnapshotter<Mesh> (util/snapshot/VtkSnapshotter.hpp:12-86): one .vts per
/// snapshot under snapshots[/outDir]/vtk/.
template <int D>
class VtkSnapshotter : public Snapshotter {
public:
	explicit VtkSnapshotter(const Task& task)
	    : Snapshotter(task), quantitiesToSnap(task.vtkSnapshotter.quantitiesToSnap) {}

protected:
	void snapshotImpl(const AbstractGrid* mesh, const int step) override;

private:
	const std::vector<PhysicalQuantities::T> quantitiesToSnap;
};

/// SliceSnapshotter<Mesh> (util/snapshot/SliceSnapshotter.hpp:12-118): velocity
/// along the last axis through the centre into snapshots/../zaxis/*.txt, and the
/// mean detector quantity over the top face (last axis) into ../detector/*.txt.
template <int D>
class SliceSnapshotter : public Snapshotter {
public:
	explicit SliceSnapshotter(const Task& task);

protected:
	void snapshotImpl(const AbstractGrid* mesh, const int step) override;

private:
	size_t gridId;
	std::vector<real> times, seismo;
	std::shared_ptr<Area> detectionArea;
	PhysicalQuantities::T quantityToWrite;
};

/// engine/cubic/AbstractFactory.hpp:22-54
template <int D>
class AbstractFactoryBase {
public:
	virtual ~AbstractFactoryBase() = default;
	virtual std::shared_ptr<AbstractMesh<D>> createMesh(
	    const Task& task, size_t gridId, const typename CubicGrid<D>::ConstructionPack& cp,
	    size_t numberOfNextPdeTimeLayers) = 0;
	virtual std::shared_ptr<GridCharacteristicMethodBase> createGcm(const Task& task) = 0;
	virtual std::shared_ptr<AbstractBorderConditions> createBorder(
	    const Task& task, std::shared_ptr<AbstractMesh<D>> mesh) = 0;
	virtual std::shared_ptr<AbstractOde> createOde(const Odes::T type) = 0;
	virtual std::shared_ptr<Snapshotter> createSnapshotter(const Task& task,
	                                                       const Snapshotters::T type) = 0;
};

/// AbstractFactory<ElasticModel<D>, CubicGrid<D>, IsotropicMaterial, HipMesh>
template <int D>
class HipFactory : public AbstractFactoryBase<D> {
public:
	explicit HipFactory(int device_) : device(device_) {}
	std::shared_ptr<AbstractMesh<D>> createMesh(const Task& task, size_t gridId,
	                                            const typename CubicGrid<D>::ConstructionPack& cp,
	                                            size_t) override {
		return std::make_shared<HipMesh<D>>(task, gridId, cp, device);
	}
	std::shared_ptr<GridCharacteristicMethodBase> createGcm(const Task& task) override {
		return std::make_shared<HipGridCharacteristicMethod<D>>(task);
	}
	std::shared_ptr<AbstractBorderConditions> createBorder(
	    const Task& task, std::shared_ptr<AbstractMesh<D>> mesh) override {
		return std::make_shared<HipBorderConditions<D>>(
		    task, dynamic_cast<const HipMesh<D>&>(*mesh));
	}
	/// AbstractFactory.hpp:90-93: every ODE type maps to MaxwellViscosityOde there;
	/// the other two do not compile in the reference (Ode.hpp:50, 75), so they are
	/// refused here.
	std::shared_ptr<AbstractOde> createOde(const Odes::T type) override {
		if (type != Odes::T::MAXWELL_VISCOSITY)
			throw Exception("only the Maxwell viscosity ODE is on this path");
		return std::make_shared<HipMaxwellViscosityOde<D>>();
	}
	/// AbstractFactory.hpp:95-105
	std::shared_ptr<Snapshotter> createSnapshotter(const Task& task,
	                                               const Snapshotters::T type) override {
		switch (type) {
		case Snapshotters::T::VTK: return std::make_shared<VtkSnapshotter<D>>(task);
		case Snapshotters::T::SLICESNAP: return std::make_shared<SliceSnapshotter<D>>(task);
		default: throw Exception("Unknown or unsupported snapshotter");
		}
	}

private:
	int device;
};

/// cubic::Engine<D> (engine/cubic/Engine.{hpp,cpp})
template <int D>
class Engine : public AbstractEngine {
public:
	typedef CubicGrid<D> Grid;
	explicit Engine(const Task& task, int device = 0);
	std::shared_ptr<const HipMesh<D>> getMesh(size_t gridId) const;

protected:
	void nextTimeStep() override;
	real estimateTimeStep() override;
	void writeSnapshots(const int step) override;

private:
	struct Body {
		std::shared_ptr<AbstractFactoryBase<D>> factory;
		std::shared_ptr<AbstractMesh<D>> mesh;
		std::shared_ptr<HipMesh<D>> stack;  // the stack this body belongs to (HipMesh::joinStack)
		bool stackLead = false;             // the member that steps the stack
		std::shared_ptr<GridCharacteristicMethodBase> gcm;
		std::shared_ptr<AbstractBorderConditions> border;
		struct Contact {
			size_t neighborId;
			int direction;
			std::shared_ptr<HipContactCopier<D>> copier;
		};
		std::vector<Contact> contacts;
		std::vector<std::shared_ptr<AbstractOde>> odes;
		std::vector<std::shared_ptr<Snapshotter>> snapshotters;
	};
	std::vector<Body> bodies;
	std::map<size_t, std::vector<size_t>> stackOrder_;  // lead id -> member ids along the stack axis
	int device;
	Body& getBody(size_t id);
	const Body& getBody(size_t id) const;
	void createGridsAndContacts(const Task& task);
	void buildStacks(const Task& task);
	/// The mesh a body's step runs on: its own, its stack's (the lead member), or
	/// none (the other members of a stack).
	HipMesh<D>* unitMesh(Body& b);
	void applyOdes();
};

}  // namespace cubic

/// engine/EngineFactory.hpp:11-38 (cubic only on this path)
std::shared_ptr<AbstractEngine> createEngine(const Task& task, int device = 0);

}  // namespace gcm
