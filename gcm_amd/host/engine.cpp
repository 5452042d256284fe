// engine.cpp -- host mirror of the cubic engine (see engine.hpp for the map).
#include "engine.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>

namespace gcm {

real Clock::time = 0;
real Clock::timeStep = 0;

void gcmxCheck(gcmx_status s, const char* what) {
	if (s != GCMX_OK)
		throw Exception(std::string(what) + ": " + gcmx_status_string(s) + ": " + gcmx_last_error());
}

// ------------------------------------------------------------ AbstractEngine --

AbstractEngine::AbstractEngine(const Task& task)
    : CourantNumber(task.globalSettings.CourantNumber) {
	Clock::setZero();
}

// AbstractEngine.cpp:18-27
void AbstractEngine::afterConstruction(const Task& task) {
	Clock::timeStep = estimateTimeStep();
	requiredTime = Clock::TimeStep() * task.globalSettings.numberOfSnaps *
	               task.globalSettings.stepsPerSnap;
	if (task.globalSettings.numberOfSnaps <= 0) requiredTime = task.globalSettings.requiredTime;
	if (!(requiredTime > 0)) throw Exception("requiredTime must be > 0");
}

// AbstractEngine.cpp:30-46
void AbstractEngine::run() {
	int step = 0;
	writeSnapshots(step);
	while (Clock::Time() < requiredTime) {
		Clock::timeStep = estimateTimeStep();
		nextTimeStep();
		step++;
		steps++;
		Clock::tickTack();
		writeSnapshots(step);
	}
}

void AbstractEngine::runSteps(int n) {
	for (int i = 0; i < n; i++) {
		Clock::timeStep = estimateTimeStep();
		nextTimeStep();
		steps++;
		Clock::tickTack();
	}
}

namespace cubic {

// ------------------------------------------------------------------ CubicGrid --

template <int D>
CubicGrid<D>::CubicGrid(size_t id_, const ConstructionPack& cp)
    : id(id_), borderSize(cp.borderSize), sizes(cp.sizes), start(cp.start), h(cp.h) {
	// CubicGrid.hpp:184-199 and calculateIndexMaker :202-225
	if (!(borderSize > 0)) throw Exception("CubicGrid: borderSize must be > 0");
	for (int i = 0; i < D; i++) {
		if (!(sizes[i] >= borderSize)) throw Exception("CubicGrid: sizes must be >= borderSize");
		if (!(h[i] > 0)) throw Exception("CubicGrid: h must be > 0");
	}
	const long long b2 = 2LL * borderSize;
	if (D == 1) {
		indexMaker[0] = 1;
	} else if (D == 2) {
		indexMaker[0] = b2 + sizes[D - 1];
		indexMaker[D - 1] = 1;
	} else {
		indexMaker[0] = (b2 + sizes[1 % D]) * (b2 + sizes[D - 1]);
		indexMaker[1 % D] = b2 + sizes[D - 1];
		indexMaker[D - 1] = 1;
	}
}

template <int D>
real CubicGrid<D>::getMinimalSpatialStep() const {
	real ans = std::numeric_limits<real>::max();
	for (int i = 0; i < D; i++)
		if (ans > h[i]) ans = h[i];
	return ans;
}

template <int D>
std::pair<typename CubicGrid<D>::IntD, typename CubicGrid<D>::IntD> CubicGrid<D>::aabb() const {
	IntD mx;
	for (int i = 0; i < D; i++) mx[i] = start[i] + sizes[i] - 1;
	return {start, mx};
}

/// Calls f(it) for every inner node in SlowXFastZ order (linal/Multiindex.hpp:99-118),
/// optionally restricted to it[axis] == fixed.
template <int D, class F>
static void forEachInner(const std::array<int, D>& sizes, F f, int axis = -1, int fixed = 0) {
	std::array<int, D> it{};
	std::array<int, D> lo{}, hi = sizes;
	if (axis >= 0) {
		lo[axis] = fixed;
		hi[axis] = fixed + 1;
	}
	it = lo;
	while (true) {
		f(it);
		int d = D - 1;
		for (; d >= 0; d--) {
			if (++it[d] < hi[d]) break;
			it[d] = lo[d];
		}
		if (d < 0) break;
	}
}

// -------------------------------------------------------------------- HipMesh --

template <int D>
HipMesh<D>::HipMesh(const Task&, size_t id_, const typename CubicGrid<D>::ConstructionPack& cp,
                    int device_)
    : AbstractMesh<D>(id_, cp), device(device_) {
	gcmx_grid_desc desc{};
	desc.dim = D;
	desc.border_size = cp.borderSize;
	for (int i = 0; i < 3; i++) {
		desc.sizes[i] = i < D ? cp.sizes[i] : 1;
		desc.start[i] = i < D ? cp.start[i] : 0;
		desc.h[i] = i < D ? cp.h[i] : 0;
	}
	gcmxCheck(gcmx_create(&desc, device, &ctx_), "gcmx_create");
}

template <int D>
HipMesh<D>::~HipMesh() {
	if (ownsCtx_) gcmx_destroy(ctx_);
}

// ---------------------------------------------------------------------- stacks --

/// Calls f(it) for every node of a grid of `sizes` INCLUDING bs ghost layers.
template <int D, class F>
static void forEachAll(const std::array<int, D>& sizes, int bs, F f) {
	std::array<int, D> it;
	for (int d = 0; d < D; d++) it[d] = -bs;
	while (true) {
		f(it);
		int d = D - 1;
		for (; d >= 0; d--) {
			if (++it[d] < sizes[d] + bs) break;
			it[d] = -bs;
		}
		if (d < 0) break;
	}
}

template <int D>
void HipMesh<D>::joinStack(const std::shared_ptr<HipMesh<D>>& stack, int axis, int offset) {
	if (stack_) throw Exception("the body is in a stack already");
	if (ownsCtx_) gcmx_destroy(ctx_);  // its device layers live in the stack
	ctx_ = stack->ctx_;
	ownsCtx_ = false;
	stack_ = stack;
	stackAxis_ = axis;
	stackOffset_ = offset;
}

template <int D>
HostState<D> HipMesh<D>::setUpMember(const Task& task) {
	if (pdeIsSetUp) throw Exception("setUpPde called twice");
	pdeIsSetUp = true;
	HostState<D> st = buildHostState<D>(task, *this);
	matrices = st.matrices;
	maximalEigenvalue = st.maximalEigenvalue;
	materialNumbers_ = st.materialNumber;
	if (matrices.size() > 1) matIdAll_ = st.matId;
	return st;
}

template <int D>
void HipMesh<D>::setUpStack(const std::vector<std::shared_ptr<HipMesh<D>>>& members,
                            const std::vector<HostState<D>>& states) {
	if (pdeIsSetUp) throw Exception("setUpPde called twice");
	pdeIsSetUp = true;
	// one table over the members' material conditions; bitwise-equal ones shared
	// (a stack of one material stays homogeneous: the non-HET one-pass step)
	std::vector<const GcmMatrices<D>*> table;
	std::vector<real> tau0;
	std::vector<std::vector<int>> remap(members.size());
	for (size_t k = 0; k < members.size(); k++)
		for (size_t c = 0; c < states[k].matrices.size(); c++) {
			const GcmMatrices<D>& m = states[k].matrices[c];
			int found = -1;
			for (size_t t = 0; t < table.size() && found < 0; t++)
				if (std::memcmp(table[t], &m, sizeof(m)) == 0 && std::memcmp(&tau0[t], &states[k].tau0[c], sizeof(real)) == 0)
					found = (int)t;
			if (found < 0) {
				found = (int)table.size();
				table.push_back(&m);
				tau0.push_back(states[k].tau0[c]);
			}
			remap[k].push_back(found);
		}
	if (table.size() > 255) throw Exception("a stack holds at most 255 materials");
	// the stack's all-nodes state: every member's inner nodes and its ghost layers
	// on the other axes; along the stack axis a member's ghost layers at a contact
	// are its neighbour's inner layers (the stack's own ghosts only at its ends)
	const int bs = this->borderSize, a = members.empty() ? 0 : members[0]->stackAxis_;
	std::vector<real> pde((size_t)this->sizeOfAllNodes() * M, 0.0);
	std::vector<uint8_t> ids((size_t)this->sizeOfAllNodes(), 0);
	std::vector<int> used(table.size(), 0);
	for (size_t k = 0; k < members.size(); k++) {
		const HipMesh<D>& mb = *members[k];
		forEachAll<D>(mb.sizes, bs, [&](const IntD& it) {
			if ((it[a] < 0 && k > 0) || (it[a] >= mb.sizes[a] && k + 1 < members.size())) return;
			IntD is = it;
			is[a] += mb.stackOffset_;
			const size_t src = (size_t)mb.getIndex(it), dst = (size_t)this->getIndex(is);
			for (int c = 0; c < M; c++) pde[dst * M + c] = states[k].pde[src * M + c];
			const int t = remap[k][states[k].matId[src]];
			ids[dst] = (uint8_t)t;
			bool inner = true;
			for (int d = 0; d < D; d++) inner = inner && it[d] >= 0 && it[d] < mb.sizes[d];
			if (inner) used[(size_t)t] = 1;
		});
	}
	std::vector<int> dev(table.size(), -1);
	int nUsed = 0;
	for (size_t t = 0; t < table.size(); t++)
		if (used[t]) dev[t] = nUsed++;
	std::vector<real> U((size_t)nUsed * D * M * M), U1(U.size()), L((size_t)nUsed * D * M);
	deviceTau0_.assign(nUsed, 0);
	maximalEigenvalue = 0;
	for (size_t t = 0; t < table.size(); t++) {
		if (dev[t] < 0) continue;
		deviceTau0_[dev[t]] = tau0[t];
		maximalEigenvalue = std::fmax(maximalEigenvalue, table[t]->getMaximalEigenvalue());
		for (int s = 0; s < D; s++) {
			const size_t o = ((size_t)dev[t] * D + s);
			std::copy(table[t]->m[s].U.begin(), table[t]->m[s].U.end(), U.begin() + o * M * M);
			std::copy(table[t]->m[s].U1.begin(), table[t]->m[s].U1.end(), U1.begin() + o * M * M);
			std::copy(table[t]->m[s].L.begin(), table[t]->m[s].L.end(), L.begin() + o * M);
		}
	}
	gcmxCheck(gcmx_set_materials(ctx_, nUsed, U.data(), U1.data(), L.data()), "gcmx_set_materials");
	if (nUsed > 1) {
		for (auto& m : ids) m = (uint8_t)std::max(0, dev[m]);
		gcmxCheck(gcmx_set_material_ids(ctx_, ids.data()), "gcmx_set_material_ids");
	}
	gcmxCheck(gcmx_upload(ctx_, pde.data()), "gcmx_upload");
}

template <int D>
typename CubicGrid<D>::ConstructionPack constructionPack(const Task& task, size_t id) {
	typename CubicGrid<D>::ConstructionPack cp;
	cp.borderSize = task.cubicGrid.borderSize;
	if ((int)task.cubicGrid.h.size() != D) throw Exception("h has the wrong size");
	const auto& cube = task.cubicGrid.cubics.at(id);
	if ((int)cube.sizes.size() != D || (int)cube.start.size() != D)
		throw Exception("cube sizes/start have the wrong size");
	for (int i = 0; i < D; i++) {
		cp.h[i] = task.cubicGrid.h[i];
		cp.sizes[i] = cube.sizes[i];
		cp.start[i] = cube.start[i];
	}
	return cp;
}

// DefaultMesh::setUpPde's host half (DefaultMesh.hpp:60-66): everything before
// the data would be stored, without touching a GPU.
template <int D>
HostState<D> buildHostState(const Task& task, const CubicGrid<D>& grid) {
	constexpr int M = pdeSize(D);
	HostState<D> st;
	const long long nAll = grid.sizeOfAllNodes();
	st.pde.assign((size_t)nAll * M, 0.0);
	st.matId.assign((size_t)nAll, 0);
	auto& pde = st.pde;
	auto& matId = st.matId;
	auto& matrices = st.matrices;

	// ---- MaterialsCondition::apply (util/task/MaterialsCondition.hpp:23-36, 70-91)
	std::vector<std::pair<std::shared_ptr<Area>, std::shared_ptr<IsotropicMaterial>>> conds;
	const auto& mc = task.materialConditions;
	if (mc.type == Task::MaterialCondition::Type::BY_AREAS) {
		conds.push_back({std::make_shared<InfiniteArea>(), mc.byAreas.defaultMaterial});
		for (const auto& m : mc.byAreas.materials) conds.push_back({m.area, m.material});
	} else {
		conds.push_back({std::make_shared<InfiniteArea>(), mc.byBodies.bodyMaterialMap.at(grid.id)});
	}
	if (conds.size() > 255) throw Exception("at most 255 material conditions per body");
	matrices.assign(conds.size(), GcmMatrices<D>());
	st.tau0.assign(conds.size(), 0);
	for (size_t c = 0; c < conds.size(); c++) {
		if (!conds[c].second) throw Exception("material condition without a material");
		ElasticModel<D>::constructGcmMatrices(matrices[c], *conds[c].second);
		st.tau0[c] = conds[c].second->tau0;
		st.materialNumber.push_back(conds[c].second->materialNumber);
	}
	forEachInner<D>(grid.sizes, [&](const std::array<int, D>& it) {
		const Real3 x = grid.coords(it);
		for (size_t c = 0; c < conds.size(); c++)
			if (conds[c].first->contains(x)) matId[(size_t)grid.getIndex(it)] = (uint8_t)c;
	});
	st.maximalEigenvalue = 0;
	for (const auto& m : matrices)
		st.maximalEigenvalue = std::fmax(st.maximalEigenvalue, m.getMaximalEigenvalue());

	// ---- InitialCondition::apply (util/task/InitialCondition.hpp:23-88)
	std::vector<std::pair<std::shared_ptr<Area>, std::array<real, M>>> ics;
	for (const auto& v : task.initialCondition.vectors) {
		if ((int)v.list.size() != M) throw Exception("initial vector has the wrong size");
		std::array<real, M> a{};
		std::copy(v.list.begin(), v.list.end(), a.begin());
		ics.push_back({v.area, a});
	}
	{
		GcmMatrices<D> front;  // mcConditions.front().material
		ElasticModel<D>::constructGcmMatrices(front, *conds.front().second);
		for (const auto& w : task.initialCondition.waves) {
			if (!(w.direction >= 0 && w.direction < D)) throw Exception("wave direction out of range");
			const int col = waveColumn(D, w.waveType);
			std::array<real, M> tmp{};
			for (int r = 0; r < M; r++) tmp[r] = front.m[w.direction].U1[r * M + col];
			const real current = getQuantity(D, w.quantity, tmp.data());
			if (current == 0) throw Exception("wave calibration quantity is zero");
			const real f = w.quantityValue / current;
			for (int r = 0; r < M; r++) tmp[r] *= f;
			ics.push_back({w.area, tmp});
		}
	}
	for (const auto& q : task.initialCondition.quantities) {
		std::array<real, M> tmp{};
		setQuantity(D, q.physicalQuantity, q.value, tmp.data());
		ics.push_back({q.area, tmp});
	}
	forEachInner<D>(grid.sizes, [&](const std::array<int, D>& it) {
		const Real3 x = grid.coords(it);
		real* v = &pde[(size_t)grid.getIndex(it) * M];
		for (int c = 0; c < M; c++) v[c] = 0;
		for (const auto& ic : ics)
			if (ic.first->contains(x))
				for (int c = 0; c < M; c++) v[c] += ic.second[c];
	});
	return st;
}

template <int D>
void HipMesh<D>::setUpPde(const Task& task) {
	if (pdeIsSetUp) throw Exception("setUpPde called twice");
	pdeIsSetUp = true;
	HostState<D> st = buildHostState<D>(task, *this);
	matrices = st.matrices;
	maximalEigenvalue = st.maximalEigenvalue;
	auto& matId = st.matId;
	materialNumbers_ = st.materialNumber;
	if (matrices.size() > 1) matIdAll_ = matId;  // before the device remap below

	// ---- device tables: only the materials the nodes actually use
	std::vector<int> used(matrices.size(), 0);
	forEachInner<D>(this->sizes, [&](const IntD& it) { used[matId[(size_t)this->getIndex(it)]] = 1; });
	std::vector<int> remap(matrices.size(), -1);
	int nUsed = 0;
	for (size_t c = 0; c < matrices.size(); c++)
		if (used[c]) remap[c] = nUsed++;
	std::vector<real> U((size_t)nUsed * D * M * M), U1(U.size()), L((size_t)nUsed * D * M);
	deviceTau0_.assign(nUsed, 0);
	for (size_t c = 0; c < matrices.size(); c++) {
		if (remap[c] < 0) continue;
		deviceTau0_[remap[c]] = st.tau0[c];
		for (int s = 0; s < D; s++) {
			const size_t o = ((size_t)remap[c] * D + s);
			std::copy(matrices[c].m[s].U.begin(), matrices[c].m[s].U.end(), U.begin() + o * M * M);
			std::copy(matrices[c].m[s].U1.begin(), matrices[c].m[s].U1.end(), U1.begin() + o * M * M);
			std::copy(matrices[c].m[s].L.begin(), matrices[c].m[s].L.end(), L.begin() + o * M);
		}
	}
	gcmxCheck(gcmx_set_materials(ctx_, nUsed, U.data(), U1.data(), L.data()), "gcmx_set_materials");
	if (nUsed > 1) {
		for (auto& m : matId) m = (uint8_t)std::max(0, remap[m]);
		gcmxCheck(gcmx_set_material_ids(ctx_, matId.data()), "gcmx_set_material_ids");
	}
	gcmxCheck(gcmx_upload(ctx_, st.pde.data()), "gcmx_upload");
}

template <int D>
std::vector<real> HipMesh<D>::pdeAll() const {
	std::vector<real> out((size_t)this->sizeOfAllNodes() * M);
	if (stack_) {  // this member's part of the stack (its ghost layers at a contact:
		           // the neighbour's inner layers, as the contact copy leaves them)
		const std::vector<real> all = stack_->pdeAll();
		const int bs = this->borderSize;
		forEachAll<D>(this->sizes, bs, [&](const IntD& it) {
			IntD is = it;
			is[stackAxis_] += stackOffset_;
			const size_t src = (size_t)stack_->getIndex(is), dst = (size_t)this->getIndex(it);
			for (int c = 0; c < M; c++) out[dst * M + c] = all[src * M + c];
		});
		return out;
	}
	gcmxCheck(gcmx_download(ctx_, out.data()), "gcmx_download");
	return out;
}

template <int D>
std::array<real, HipMesh<D>::M> HipMesh<D>::pde(const IntD& it) const {
	const std::vector<real> all = pdeAll();
	std::array<real, M> v;
	const size_t i = (size_t)this->getIndex(it);
	for (int c = 0; c < M; c++) v[c] = all[i * M + c];
	return v;
}

// ----------------------------------------------------------------- the stage --

template <int D>
void HipGridCharacteristicMethod<D>::stage(const int s, const real& timeStep,
                                           AbstractGrid& mesh_) const {
	HipMesh<D>& mesh = dynamic_cast<HipMesh<D>&>(mesh_);  // std::bad_cast like the reference
	gcmxCheck(gcmx_stage(mesh.ctx(), s, timeStep), "gcmx_stage");
}

template <int D>
void HipGridCharacteristicMethod<D>::step(const real& timeStep, HipMesh<D>& mesh) const {
	gcmxCheck(gcmx_step(mesh.ctx(), timeStep), "gcmx_step");
}

// ------------------------------------------------------------ border conditions --

static int quantityCode(PhysicalQuantities::T q) { return static_cast<int>(q); }

template <int D>
HipBorderConditions<D>::HipBorderConditions(const Task& task, const HipMesh<D>& mesh) {
	const auto found = task.cubicBorderConditions.find(mesh.id);
	if (found == task.cubicBorderConditions.end()) {
		uniform = true;  // no face has a condition
		return;
	}
	// per face, per face node (forEachInner order): the last condition whose
	// area contains the node (later conditions overwrite the whole ghost)
	std::array<std::vector<int>, 6> effective;
	for (int f = 0; f < 2 * D; f++) {
		size_t n = 1;
		for (int d = 0; d < D; d++)
			if (d != f / 2) n *= (size_t)mesh.sizes[d];
		effective[f].assign(n, -1);
	}
	try {
		for (const auto& bc : found->second) {
			Condition c;
			c.direction = bc.direction;
			if (!(bc.direction >= 0 && bc.direction < D)) throw Exception("border direction out of range");
			for (const auto& q : bc.values) {
				if (!hasQuantity(D, q.first)) throw Exception("border quantity not in the PDE vector");
				c.values.push_back({q.first, q.second});  // std::map order == reference order
			}
			if (c.values.size() > GCMX_MAX_BORDER_Q) throw Exception("too many border quantities");
			const int index = (int)conditions.size();
			auto collect = [&](int side, std::vector<int>& out) {
				std::vector<int>& eff = effective[2 * bc.direction + side];
				size_t k = 0;
				forEachInner<D>(mesh.sizes, [&](const std::array<int, D>& it) {
					if (bc.area->contains(mesh.coords(it))) {
						for (int d = 0; d < D; d++) out.push_back(it[d]);
						eff[k] = index;
					}
					k++;
				}, bc.direction, side ? mesh.sizes[bc.direction] - 1 : 0);
			};
			collect(0, c.leftNodes);
			collect(1, c.rightNodes);
			try {
				gcmxCheck(gcmx_border_nodes_create(mesh.ctx(), c.direction, -1, (int)(c.leftNodes.size() / D),
				                                   c.leftNodes.data(), &c.leftD), "gcmx_border_nodes_create");
				gcmxCheck(gcmx_border_nodes_create(mesh.ctx(), c.direction, +1, (int)(c.rightNodes.size() / D),
				                                   c.rightNodes.data(), &c.rightD), "gcmx_border_nodes_create");
			} catch (...) {
				gcmx_border_nodes_destroy(c.leftD);
				throw;
			}
			conditions.push_back(std::move(c));
		}
	} catch (...) {  // the destructor does not run for a constructor that throws
		for (auto& done : conditions) {
			gcmx_border_nodes_destroy(done.leftD);
			gcmx_border_nodes_destroy(done.rightD);
		}
		conditions.clear();
		throw;
	}
	uniform = true;
	for (int f = 0; f < 2 * D; f++) {
		const std::vector<int>& eff = effective[f];
		for (int e : eff) uniform = uniform && e == eff[0];
		faceCondition[f] = eff.empty() ? -1 : eff[0];
	}
	const char* noMaps = std::getenv("GCMX_NO_FACE_MAPS");  // 1: node lists only
	if (!uniform && conditions.size() <= GCMX_MAX_FACE_CONDITIONS && !(noMaps && std::atoi(noMaps) != 0)) {
		// partial faces: each face node's last condition, as one byte per face node
		std::array<std::vector<uint8_t>, 6> maps;
		const uint8_t* ptr[6] = {};
		for (int f = 0; f < 2 * D; f++) {
			maps[f].resize(effective[f].size());
			for (size_t k = 0; k < effective[f].size(); k++)
				maps[f][k] = effective[f][k] < 0 ? (uint8_t)GCMX_NO_FACE_CONDITION : (uint8_t)effective[f][k];
			ptr[f] = maps[f].data();
		}
		if (gcmx_face_map_create(mesh.ctx(), ptr, &faceMap_) != GCMX_OK) {
			// the map only lets the one-pass step take the partial faces: without
			// it the conditions' node lists (above) still serve every stage, so the
			// engine runs on the per-stage path
			std::fprintf(stderr, "gcm_amd: gcmx_face_map_create failed (%s); partial faces run on the per-stage path\n",
			             gcmx_last_error());
			faceMap_ = nullptr;
		}
	}
}

template <int D>
int HipBorderConditions<D>::conditionsAt(gcmx_face* out) const {
	for (size_t k = 0; k < conditions.size(); k++) {
		const Condition& c = conditions[k];
		out[k] = gcmx_face{};
		out[k].enabled = 1;
		out[k].n_quantities = (int)c.values.size();
		for (size_t i = 0; i < c.values.size(); i++) {
			out[k].quantities[i] = quantityCode(c.values[i].first);
			out[k].values[i] = c.values[i].second(Clock::Time());
		}
	}
	return (int)conditions.size();
}

template <int D>
HipBorderConditions<D>::~HipBorderConditions() {
	gcmx_face_map_destroy(faceMap_);
	for (auto& c : conditions) {
		gcmx_border_nodes_destroy(c.leftD);
		gcmx_border_nodes_destroy(c.rightD);
	}
}

template <int D>
void HipBorderConditions<D>::apply(AbstractGrid& mesh_, const int direction) const {
	HipMesh<D>& mesh = dynamic_cast<HipMesh<D>&>(mesh_);
	for (const auto& c : conditions) {
		if (c.direction != direction) continue;
		std::vector<int> qs;
		std::vector<real> vals;
		for (const auto& v : c.values) {
			qs.push_back(quantityCode(v.first));
			vals.push_back(v.second(Clock::Time()));
		}
		gcmxCheck(gcmx_border_apply(mesh.ctx(), c.leftD, (int)qs.size(), qs.data(), vals.data()),
		          "gcmx_border_apply");
		gcmxCheck(gcmx_border_apply(mesh.ctx(), c.rightD, (int)qs.size(), qs.data(), vals.data()),
		          "gcmx_border_apply");
	}
}

template <int D>
void HipBorderConditions<D>::faces(gcmx_face* out) const {
	for (int f = 0; f < 2 * D; f++) {
		out[f] = gcmx_face{};
		if (faceCondition[f] < 0) continue;
		const Condition& c = conditions[(size_t)faceCondition[f]];
		out[f].enabled = 1;
		out[f].n_quantities = (int)c.values.size();
		for (size_t k = 0; k < c.values.size(); k++) {
			out[f].quantities[k] = quantityCode(c.values[k].first);
			out[f].values[k] = c.values[k].second(Clock::Time());
		}
	}
}

template <int D>
void HipContactCopier<D>::apply(HipMesh<D>& a, const HipMesh<D>& b) const {
	gcmxCheck(gcmx_copy_box(a.ctx(), dmin.data(), dmax.data(), b.ctx(), smin.data()), "gcmx_copy_box");
}

// --------------------------------------------------------------------- Engine --

template <int D>
Engine<D>::Engine(const Task& task, int device_) : AbstractEngine(task), device(device_) {
	if (task.globalSettings.dimensionality != D) throw Exception("dimensionality mismatch");
	createGridsAndContacts(task);
	buildStacks(task);
	std::map<size_t, HostState<D>> memberStates;
	for (const auto& tb : task.bodies) {
		Body& body = getBody(tb.first);
		if (body.stack)
			memberStates.emplace(tb.first, std::dynamic_pointer_cast<HipMesh<D>>(body.mesh)->setUpMember(task));
		else
			body.mesh->setUpPde(task);
		body.gcm = body.factory->createGcm(task);
		body.border = body.factory->createBorder(task, body.mesh);
		for (const Snapshotters::T snapType : task.globalSettings.snapshottersId)
			body.snapshotters.push_back(body.factory->createSnapshotter(task, snapType));
		for (const Odes::T odeType : tb.second.odes) body.odes.push_back(body.factory->createOde(odeType));
	}
	for (Body& lead : bodies) {  // every stack's set-up from its members' host states
		if (!lead.stackLead) continue;
		std::vector<std::shared_ptr<HipMesh<D>>> members;
		std::vector<HostState<D>> states;
		for (size_t id : stackOrder_.at(lead.mesh->id)) {
			members.push_back(std::dynamic_pointer_cast<HipMesh<D>>(getBody(id).mesh));
			states.push_back(std::move(memberStates.at(id)));
		}
		lead.stack->setUpStack(members, states);
	}
	afterConstruction(task);
}

template <int D>
typename Engine<D>::Body& Engine<D>::getBody(size_t id) {
	for (Body& b : bodies)
		if (b.mesh->id == id) return b;
	throw Exception("There isn't a body with given id");
}

template <int D>
const typename Engine<D>::Body& Engine<D>::getBody(size_t id) const {
	for (const Body& b : bodies)
		if (b.mesh->id == id) return b;
	throw Exception("There isn't a body with given id");
}

template <int D>
std::shared_ptr<const HipMesh<D>> Engine<D>::getMesh(size_t gridId) const {
	return std::dynamic_pointer_cast<const HipMesh<D>>(getBody(gridId).mesh);
}

// Engine.cpp:38-87 (factory choice: Engine.cpp:155-189)
template <int D>
void Engine<D>::createGridsAndContacts(const Task& task) {
	if (task.bodies.empty()) throw Exception("the task has no bodies");
	if (task.bodies.size() != task.cubicGrid.cubics.size())
		throw Exception("every body needs a cube");
	for (const auto& tb : task.bodies) {
		if (tb.second.materialId != Materials::T::ISOTROPIC || tb.second.modelId != Models::T::ELASTIC)
			throw Exception("only isotropic elastic bodies are on this path");
		Body body;
		body.factory = std::make_shared<HipFactory<D>>(device);
		const auto cp = constructionPack<D>(task, tb.first);
		body.mesh = body.factory->createMesh(task, tb.first, cp, 1);
		bodies.push_back(body);
	}
	for (Body& body : bodies) {
		for (const Body& other : bodies) {
			if (other.mesh->id == body.mesh->id) continue;
			auto a = body.mesh->aabb(), b = other.mesh->aabb();
			std::array<int, D> mn, mx, w;
			bool valid = true;
			for (int i = 0; i < D; i++) {
				mn[i] = std::max(a.first[i], b.first[i]);
				mx[i] = std::min(a.second[i], b.second[i]);
				w[i] = mx[i] - mn[i];
				if (w[i] < 0) valid = false;
			}
			if (valid) throw Exception("Bodies must not intersect");
			int axis = 0;
			int minW = w[0];
			for (int i = 1; i < D; i++)
				if (w[i] < minW) {
					axis = i;
					minW = w[i];
				}
			if (minW != -1) continue;  // no contact
			std::array<int, D> bmin = mn, bmax = mx;
			if (body.mesh->start[axis] > other.mesh->start[axis]) bmin[axis] -= body.mesh->borderSize;
			else bmax[axis] += body.mesh->borderSize;
			std::array<int, 3> dmin{0, 0, 0}, dmax{1, 1, 1}, smin{0, 0, 0};
			for (int i = 0; i < D; i++) {
				dmin[i] = bmin[i] - body.mesh->start[i];
				dmax[i] = bmax[i] - body.mesh->start[i] + 1;
				smin[i] = bmin[i] - other.mesh->start[i];
			}
			typename Body::Contact contact;
			contact.neighborId = other.mesh->id;
			contact.direction = axis;
			contact.copier = std::make_shared<HipContactCopier<D>>(dmin, dmax, smin);
			body.contacts.push_back(contact);
		}
	}
}

// Stacks (HipMesh::joinStack): chains of 3-D bodies along one axis whose every
// contact lies along that axis, between bodies of equal sizes and starts on the
// other two axes, with no border conditions and the same ODEs.  Their contact
// copies then only ever write what the stack's own stages read, so the chain
// runs as one grid: one launch of the one-pass step over all its nodes (along
// x the separate bodies could take the one-pass step too, but each as a thin
// launch with short y chunks, plus the contact copies: 256^3 as 4 x-bodies
// 0.86 ms/step against 0.57 as one grid).  The inner nodes are the separate
// bodies' bitwise; ghost layers at a contact hold the neighbour's current inner
// nodes instead of the copy made before the last stage (scratch: no output
// reads them).  GCMX_NO_STACKS=1 keeps the separate bodies (A/B, tests).
template <int D>
void Engine<D>::buildStacks(const Task& task) {
	if (D != 3) return;
	if (const char* e = std::getenv("GCMX_NO_STACKS"))
		if (std::atoi(e) != 0) return;
	auto hasBorder = [&](size_t id) {
		const auto f = task.cubicBorderConditions.find(id);
		return f != task.cubicBorderConditions.end() && !f->second.empty();
	};
	for (int a = 0; a < D; a++) {
		std::map<size_t, bool> ok;  // every contact along a, partners of equal cross-section
		for (Body& b : bodies) {
			bool good = !b.stack && !b.contacts.empty() && !hasBorder(b.mesh->id);
			for (const auto& c : b.contacts) {
				if (c.direction != a) good = false;
				const Body& o = getBody(c.neighborId);
				for (int d = 0; d < D; d++)
					if (d != a && (o.mesh->sizes[d] != b.mesh->sizes[d] || o.mesh->start[d] != b.mesh->start[d]))
						good = false;
			}
			ok[b.mesh->id] = good;
		}
		std::map<size_t, bool> seen;
		for (Body& b : bodies) {
			const size_t id0 = b.mesh->id;
			if (!ok[id0] || seen[id0]) continue;
			std::vector<size_t> comp, todo{id0};
			seen[id0] = true;
			bool allGood = true;
			while (!todo.empty()) {  // the bodies connected to id0 by contacts
				const size_t id = todo.back();
				todo.pop_back();
				comp.push_back(id);
				for (const auto& c : getBody(id).contacts) {
					if (!ok[c.neighborId]) allGood = false;
					if (!seen[c.neighborId]) {
						seen[c.neighborId] = true;
						todo.push_back(c.neighborId);
					}
				}
			}
			if (!allGood || comp.size() < 2) continue;
			std::sort(comp.begin(), comp.end(),
			          [&](size_t p, size_t q) { return getBody(p).mesh->start[a] < getBody(q).mesh->start[a]; });
			bool chain = true;
			int total = 0;
			for (size_t k = 0; k < comp.size(); k++) {
				const auto& m = *getBody(comp[k]).mesh;
				if (k > 0) {
					const auto& p = *getBody(comp[k - 1]).mesh;
					chain = chain && m.start[a] == p.start[a] + p.sizes[a];
					chain = chain && task.bodies.at(comp[k]).odes == task.bodies.at(comp[0]).odes;
				}
				total += m.sizes[a];
			}
			if (!chain) continue;
			auto cp = constructionPack<D>(task, comp[0]);
			cp.sizes[a] = total;
			auto stack = std::make_shared<HipMesh<D>>(task, comp[0], cp, device);
			int off = 0;
			for (size_t id : comp) {
				Body& m = getBody(id);
				auto hm = std::dynamic_pointer_cast<HipMesh<D>>(m.mesh);
				hm->joinStack(stack, a, off);
				off += hm->sizes[a];
				m.stack = stack;
				m.contacts.clear();  // inside the stack: its own rows
			}
			getBody(comp[0]).stackLead = true;
			stackOrder_[comp[0]] = comp;
		}
	}
}

template <int D>
HipMesh<D>* Engine<D>::unitMesh(Body& b) {
	if (b.stack) return b.stackLead ? b.stack.get() : nullptr;
	return &dynamic_cast<HipMesh<D>&>(*b.mesh);
}

// Engine.cpp:90-121
template <int D>
void Engine<D>::nextTimeStep() {
	bool plain = true, faces = true, xcontacts = D == 3;
	for (const Body& b : bodies) {
		plain = plain && b.border->empty() && b.contacts.empty();
		faces = faces && (b.border->uniformFaces() || b.border->faceMap()) && b.contacts.empty();
		xcontacts = xcontacts && b.border->empty();
		for (const auto& contact : b.contacts) xcontacts = xcontacts && contact.direction == 0;
	}
	// A body whose only ODE is MaxwellViscosityOde hands it to the library with
	// the step (gcmx_step_ode): the same results as the stages followed by the ODE
	// (Engine.cpp:115-119), in one pass over the layer where the step is fused.
	auto oneMaxwell = [](const Body& b) {
		return b.odes.size() == 1 && dynamic_cast<const HipMaxwellViscosityOde<D>*>(b.odes[0].get()) != nullptr;
	};
	if (plain || xcontacts) {
		// No border or contact work between the stages: one gcmx_step per body
		// (identical results; lets the library use its fused kernels).  3-D
		// bodies whose contacts all lie along x: every ContactCopier of the step
		// runs before stage 0 and reads the neighbours' layer E_n
		// (Engine.cpp:99-107), and only stage 0 reads x ghosts, so all copies go
		// first, then one gcmx_step per body (the x-ghost copy keeps the
		// one-pass step admissible, gcmx_copy_box).
		if (!plain)
			for (Body& body : bodies)
				for (auto& contact : body.contacts)
					contact.copier->apply(dynamic_cast<HipMesh<D>&>(*body.mesh),
					                      dynamic_cast<const HipMesh<D>&>(*getBody(contact.neighborId).mesh));
		for (Body& b : bodies) {
			HipMesh<D>* um = unitMesh(b);
			if (!um) continue;  // a stack member stepped by its lead
			HipMesh<D>& mesh = *um;
			if (oneMaxwell(b)) {
				const auto& tau0 = mesh.deviceTau0();
				gcmxCheck(gcmx_step_ode(mesh.ctx(), Clock::TimeStep(), nullptr, tau0.data(), (int)tau0.size()),
				          "gcmx_step_ode");
				continue;
			}
			std::static_pointer_cast<HipGridCharacteristicMethod<D>>(b.gcm)->step(Clock::TimeStep(), mesh);
			for (auto& ode : b.odes) ode->apply(mesh, Clock::TimeStep());
		}
		return;
	}
	if (faces) {
		// Whole-face border conditions and no contacts: every stage's
		// BorderConditions::apply is a function of the face only, so the library
		// runs the step (fused where admissible) with the faces' values at
		// Clock::Time() -- the time all D stages of the reference step see.
		for (Body& b : bodies) {
			HipMesh<D>* um = unitMesh(b);
			if (!um) continue;
			HipMesh<D>& mesh = *um;
			if (const gcmx_face_map* fm = b.border->faceMap()) {
				// partial faces: each face node's own last condition, the whole step in
				// the library (one pass where admissible), then the ODEs
				gcmx_face conds[GCMX_MAX_FACE_CONDITIONS];
				const int n = b.border->conditionsAt(conds);
				gcmxCheck(gcmx_step_face_map(mesh.ctx(), Clock::TimeStep(), fm, n, conds), "gcmx_step_face_map");
				for (auto& ode : b.odes) ode->apply(mesh, Clock::TimeStep());
				continue;
			}
			gcmx_face f[6];
			b.border->faces(f);
			if (oneMaxwell(b)) {
				const auto& tau0 = mesh.deviceTau0();
				gcmxCheck(gcmx_step_ode(mesh.ctx(), Clock::TimeStep(), f, tau0.data(), (int)tau0.size()),
				          "gcmx_step_ode");
				continue;
			}
			gcmxCheck(gcmx_step_faces(mesh.ctx(), Clock::TimeStep(), f), "gcmx_step_faces");
			for (auto& ode : b.odes) ode->apply(mesh, Clock::TimeStep());
		}
		return;
	}
	for (int stage = 0; stage < D; stage++) {
		for (Body& body : bodies) body.border->apply(*body.mesh, stage);
		for (Body& body : bodies)
			for (auto& contact : body.contacts)
				if (contact.direction == stage)
					contact.copier->apply(dynamic_cast<HipMesh<D>&>(*body.mesh),
					                      dynamic_cast<const HipMesh<D>&>(*getBody(contact.neighborId).mesh));
		for (Body& body : bodies) {
			HipMesh<D>* um = unitMesh(body);
			if (!um) continue;
			body.gcm->stage(stage, Clock::TimeStep(), *um);
			um->swapCurrAndNextPdeTimeLayer(0);
		}
	}
	applyOdes();
}

// Engine.cpp:115-119: ODEs after all stages of the step.
template <int D>
void Engine<D>::applyOdes() {
	for (Body& body : bodies) {
		HipMesh<D>* um = unitMesh(body);
		if (!um) continue;
		for (auto& ode : body.odes) ode->apply(*um, Clock::TimeStep());
	}
}

template <int D>
void Engine<D>::writeSnapshots(const int step) {
	for (Body& body : bodies)
		for (auto& snap : body.snapshotters) snap->snapshot(body.mesh.get(), step);
}

// ------------------------------------------------------------- snapshotters --

template <int D>
void VtkSnapshotter<D>::snapshotImpl(const AbstractGrid* mesh_, const int step) {
	const HipMesh<D>* mesh = dynamic_cast<const HipMesh<D>*>(mesh_);
	if (!mesh) throw Exception("VtkSnapshotter: not a cubic mesh");
	const std::vector<real> pde = mesh->pdeAll();  // the one device -> host copy
	const auto& ids = mesh->materialIdsAll();
	writeVtkSnapshot<D>(makeFileNameForSnapshot(std::to_string(mesh->id), step, "vts", "vtk"),
	                    mesh->sizes, mesh->start, mesh->h, mesh->borderSize, pde.data(),
	                    ids.empty() ? nullptr : ids.data(), mesh->materialNumbers(),
	                    quantitiesToSnap);
}

template <int D>
SliceSnapshotter<D>::SliceSnapshotter(const Task& task) : Snapshotter(task) {
	if (task.detector.quantities.size() != 1)  // SliceSnapshotter.hpp:31
		throw Exception("SliceSnapshotter: exactly one detector quantity is supported");
	quantityToWrite = task.detector.quantities[0];
	detectionArea = task.detector.area;
	gridId = task.detector.gridId;
	if (!detectionArea) throw Exception("SliceSnapshotter: detector area missing");
}

template <int D>
void SliceSnapshotter<D>::snapshotImpl(const AbstractGrid* mesh_, const int step) {
	const HipMesh<D>* mesh = dynamic_cast<const HipMesh<D>*>(mesh_);
	if (!mesh) throw Exception("SliceSnapshotter: not a cubic mesh");
	constexpr int M = pdeSize(D);
	const int direction = D - 1;
	const std::vector<real> pde = mesh->pdeAll();
	auto at = [&](const std::array<int, D>& it) { return &pde[(size_t)mesh->getIndex(it) * M]; };
	// along the last axis through sizes / 2 (SliceSnapshotter.hpp:45-63)
	std::array<int, D> it;
	for (int i = 0; i < D; i++) it[i] = mesh->sizes[i] / 2;
	std::vector<real> coordZ, Vz;
	for (int k = 0; k < mesh->sizes[direction]; k++) {
		it[direction] = k;
		coordZ.push_back(mesh->coords(it)[direction]);
		Vz.push_back(at(it)[direction]);
	}
	writeColumns(makeFileNameForSnapshot(std::to_string(mesh->id), step, "txt", "zaxis"),
	             {coordZ, Vz});
	if (mesh->id != gridId) return;
	// upper detector: mean over the right border of the last axis (hpp:65-88)
	std::vector<real> valuesInArea;
	forEachInner<D>(mesh->sizes, [&](const std::array<int, D>& j) {
		if (j[direction] != mesh->sizes[direction] - 1) return;
		if (detectionArea->contains(mesh->coords(j)))
			valuesInArea.push_back(getQuantity(D, quantityToWrite, at(j)));
	});
	if (valuesInArea.empty()) throw Exception("SliceSnapshotter: no node in the detection area");
	real sum = 0;
	for (real v : valuesInArea) sum += v;  // std::accumulate order
	const real valueToWrite = sum / (real)valuesInArea.size();
	times.push_back(Clock::Time());
	seismo.push_back((precision)valueToWrite);
	writeColumns(makeFileNameForSnapshot(std::to_string(mesh->id), step, "txt", "detector"),
	             {times, seismo});
}

template <int D>
void HipMaxwellViscosityOde<D>::apply(AbstractGrid& mesh_, const real timeStep) {
	HipMesh<D>& mesh = dynamic_cast<HipMesh<D>&>(mesh_);
	const auto& tau0 = mesh.deviceTau0();
	gcmxCheck(gcmx_ode_maxwell(mesh.ctx(), timeStep, tau0.data(), (int)tau0.size()),
	          "gcmx_ode_maxwell");
}

// Engine.cpp:124-140
template <int D>
real Engine<D>::estimateTimeStep() {
	real maxEigenvalue = 0;
	const auto h = bodies.front().mesh->h;
	for (const Body& b : bodies) {
		if (!(h == b.mesh->h)) throw Exception("all bodies must share h");
		const real e = b.mesh->getMaximalEigenvalue();
		if (e > maxEigenvalue) maxEigenvalue = e;
	}
	return CourantNumber * bodies.front().mesh->getMinimalSpatialStep() / maxEigenvalue;
}

template class CubicGrid<1>;
template class CubicGrid<2>;
template class CubicGrid<3>;
template class HipMesh<1>;
template class HipMesh<2>;
template class HipMesh<3>;
template class HipGridCharacteristicMethod<1>;
template class HipGridCharacteristicMethod<2>;
template class HipGridCharacteristicMethod<3>;
template class HipBorderConditions<1>;
template class HipBorderConditions<2>;
template class HipBorderConditions<3>;
template class HipContactCopier<1>;
template class HipContactCopier<2>;
template class HipContactCopier<3>;
template class VtkSnapshotter<1>;
template class VtkSnapshotter<2>;
template class VtkSnapshotter<3>;
template class SliceSnapshotter<1>;
template class SliceSnapshotter<2>;
template class SliceSnapshotter<3>;
template class HipMaxwellViscosityOde<1>;
template class HipMaxwellViscosityOde<2>;
template class HipMaxwellViscosityOde<3>;
template CubicGrid<1>::ConstructionPack constructionPack<1>(const Task&, size_t);
template CubicGrid<2>::ConstructionPack constructionPack<2>(const Task&, size_t);
template CubicGrid<3>::ConstructionPack constructionPack<3>(const Task&, size_t);
template HostState<1> buildHostState<1>(const Task&, const CubicGrid<1>&);
template HostState<2> buildHostState<2>(const Task&, const CubicGrid<2>&);
template HostState<3> buildHostState<3>(const Task&, const CubicGrid<3>&);
template class Engine<1>;
template class Engine<2>;
template class Engine<3>;

}  // namespace cubic

// engine/EngineFactory.hpp:11-38
std::shared_ptr<AbstractEngine> createEngine(const Task& task, int device) {
	if (task.globalSettings.gridId != Grids::T::CUBIC)
		throw Exception("only the cubic engine is on this path");
	switch (task.globalSettings.dimensionality) {
	case 1: return std::make_shared<cubic::Engine<1>>(task, device);
	case 2: return std::make_shared<cubic::Engine<2>>(task, device);
	case 3: return std::make_shared<cubic::Engine<3>>(task, device);
	default: throw Exception("Invalid dimensionality");
	}
}

}  // namespace gcm
