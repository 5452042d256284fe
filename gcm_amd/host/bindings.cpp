// bindings.cpp -- pybind11 module gcm_amd._gcm_host: the C++ host mirror
// (Task / createEngine / cubic::Engine<D>) for Python tests and tools.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <type_traits>

#include "engine.hpp"
#include "simplex.hpp"
#include "../csrc/contact.hpp"

namespace py = pybind11;
using namespace gcm;

namespace {

Real3 r3(const py::sequence& s) {
	Real3 r = {0, 0, 0};
	for (size_t i = 0; i < 3 && i < (size_t)py::len(s); i++) r[i] = s[i].cast<real>();
	return r;
}

/// ("infinite",) | ("box", min3, max3) | ("sphere", r, c3) | ("cylinder", r, b3, e3)
std::shared_ptr<Area> makeArea(const py::tuple& t) {
	const std::string kind = t[0].cast<std::string>();
	if (kind == "infinite") return std::make_shared<InfiniteArea>();
	if (kind == "box") return std::make_shared<AxisAlignedBoxArea>(r3(t[1]), r3(t[2]));
	if (kind == "sphere") return std::make_shared<SphereArea>(t[1].cast<real>(), r3(t[2]));
	if (kind == "cylinder")
		return std::make_shared<StraightBoundedCylinderArea>(t[1].cast<real>(), r3(t[2]), r3(t[3]));
	throw Exception("unknown area kind " + kind);
}

PhysicalQuantities::T quantity(const std::string& q) {
	static const std::map<std::string, PhysicalQuantities::T> m = {
	    {"Vx", PhysicalQuantities::T::Vx},   {"Vy", PhysicalQuantities::T::Vy},
	    {"Vz", PhysicalQuantities::T::Vz},   {"Sxx", PhysicalQuantities::T::Sxx},
	    {"Sxy", PhysicalQuantities::T::Sxy}, {"Sxz", PhysicalQuantities::T::Sxz},
	    {"Syy", PhysicalQuantities::T::Syy}, {"Syz", PhysicalQuantities::T::Syz},
	    {"Szz", PhysicalQuantities::T::Szz}, {"PRESSURE", PhysicalQuantities::T::PRESSURE}};
	auto it = m.find(q);
	if (it == m.end()) throw Exception("unknown quantity " + q);
	return it->second;
}

Waves::T wave(const std::string& w) {
	static const std::map<std::string, Waves::T> m = {
	    {"P_FORWARD", Waves::T::P_FORWARD},   {"P_BACKWARD", Waves::T::P_BACKWARD},
	    {"S1_FORWARD", Waves::T::S1_FORWARD}, {"S1_BACKWARD", Waves::T::S1_BACKWARD},
	    {"S2_FORWARD", Waves::T::S2_FORWARD}, {"S2_BACKWARD", Waves::T::S2_BACKWARD}};
	auto it = m.find(w);
	if (it == m.end()) throw Exception("unknown wave " + w);
	return it->second;
}

/// Dimension-erased handle on cubic::Engine<D>.
struct PyEngine {
	std::shared_ptr<AbstractEngine> e;
	int D;
	template <int DD>
	cubic::Engine<DD>& as() { return dynamic_cast<cubic::Engine<DD>&>(*e); }

	py::array_t<real> pde(size_t id) {
		std::vector<real> v;
		std::vector<ssize_t> shape;
		auto grab = [&](auto& eng) {
			auto mesh = eng.getMesh(id);
			v = mesh->pdeAll();
			for (int i = 0; i < (int)mesh->sizes.size(); i++) shape.push_back(mesh->sizes[i] + 2 * mesh->borderSize);
			shape.push_back((ssize_t)(v.size() / (size_t)mesh->sizeOfAllNodes()));
		};
		if (D == 1) grab(as<1>());
		else if (D == 2) grab(as<2>());
		else grab(as<3>());
		py::array_t<real> out(shape);
		std::copy(v.begin(), v.end(), out.mutable_data());
		return out;
	}
	void runSteps(int n) { e->runSteps(n); }
	/// wait for a body's device work (timing)
	void sync(size_t id) {
		gcmx_ctx* c = nullptr;
		if (D == 1) c = as<1>().getMesh(id)->ctx();
		else if (D == 2) c = as<2>().getMesh(id)->ctx();
		else c = as<3>().getMesh(id)->ctx();
		gcmxCheck(gcmx_sync(c), "gcmx_sync");
	}
	std::string path(size_t id) {
		gcmx_ctx* c = nullptr;
		if (D == 1) c = as<1>().getMesh(id)->ctx();
		else if (D == 2) c = as<2>().getMesh(id)->ctx();
		else c = as<3>().getMesh(id)->ctx();
		static const char* names[] = {"auto", "generic", "split", "fused"};
		return names[gcmx_effective_path(c)];
	}
	/// The path the body's last step actually ran (gcmx_last_step_path).
	std::string lastPath(size_t id) {
		gcmx_ctx* c = nullptr;
		if (D == 1) c = as<1>().getMesh(id)->ctx();
		else if (D == 2) c = as<2>().getMesh(id)->ctx();
		else c = as<3>().getMesh(id)->ctx();
		static const char* names[] = {"auto", "generic", "split", "fused"};
		return names[gcmx_last_step_path(c)];
	}
	/// Whether the body's last step folded its Maxwell ODE into the one-pass step (gcmx_last_ode_fused).
	bool odeFused(size_t id) {
		gcmx_ctx* c = nullptr;
		if (D == 1) c = as<1>().getMesh(id)->ctx();
		else if (D == 2) c = as<2>().getMesh(id)->ctx();
		else c = as<3>().getMesh(id)->ctx();
		return gcmx_last_ode_fused(c) != 0;
	}
	real maximalEigenvalue(size_t id) {
		if (D == 1) return as<1>().getMesh(id)->getMaximalEigenvalue();
		if (D == 2) return as<2>().getMesh(id)->getMaximalEigenvalue();
		return as<3>().getMesh(id)->getMaximalEigenvalue();
	}
};

/// buildHostState for body `id` of `task`, as numpy arrays shaped like the grid.
template <int D>
py::dict hostState(const Task& task, size_t id) {
	cubic::CubicGrid<D> grid(id, cubic::constructionPack<D>(task, id));
	auto st = cubic::buildHostState<D>(task, grid);
	std::vector<ssize_t> shape;
	for (int i = 0; i < D; i++) shape.push_back(grid.sizes[i] + 2 * grid.borderSize);
	py::array_t<uint8_t> ids(shape);
	std::copy(st.matId.begin(), st.matId.end(), ids.mutable_data());
	shape.push_back(pdeSize(D));
	py::array_t<real> pde(shape);
	std::copy(st.pde.begin(), st.pde.end(), pde.mutable_data());
	py::dict d;
	d["pde"] = pde;
	d["mat_ids"] = ids;
	d["maximal_eigenvalue"] = st.maximalEigenvalue;
	d["n_conditions"] = st.matrices.size();
	return d;
}

/// VtkSnapshotter's file for body `id` without a GPU: the set-up layer of the
/// task, or `pde` (all nodes incl. ghosts, [..., M]) when given.
template <int D>
void writeVtkHost(const Task& task, size_t id, const std::string& fileName, py::object pde) {
	cubic::CubicGrid<D> grid(id, cubic::constructionPack<D>(task, id));
	auto st = cubic::buildHostState<D>(task, grid);
	std::vector<real> layer = st.pde;
	if (!pde.is_none()) {
		auto a = pde.cast<py::array_t<real, py::array::c_style | py::array::forcecast>>();
		if ((size_t)a.size() != layer.size()) throw Exception("write_vtk: pde has the wrong size");
		std::copy(a.data(), a.data() + a.size(), layer.begin());
	}
	makeParentDirectories(fileName);
	cubic::writeVtkSnapshot<D>(fileName, grid.sizes, grid.start, grid.h, grid.borderSize,
	                           layer.data(), st.matId.data(), st.materialNumber,
	                           task.vtkSnapshotter.quantitiesToSnap);
}

/// One body of the GPU-free simplex set-up (simplex::buildHostPlans) as numpy arrays.
py::dict simplexBodyDict(const simplex::BodyPlans& p, real tau) {
	using namespace simplex;
	const ssize_t nv = p.mesh.nVertices(), nc = (ssize_t)p.mesh.cells.size();
	py::array_t<double> coords({nv, (ssize_t)3});
	for (ssize_t i = 0; i < nv; i++)
		for (int c = 0; c < 3; c++) coords.mutable_at(i, c) = p.mesh.v[i][c];
	py::array_t<int> cells({nc, (ssize_t)4});
	for (ssize_t i = 0; i < nc; i++)
		for (int c = 0; c < 4; c++) cells.mutable_at(i, c) = p.mesh.cells[i][c];
	py::array_t<double> U({(ssize_t)3, (ssize_t)9, (ssize_t)9}), U1({(ssize_t)3, (ssize_t)9, (ssize_t)9});
	for (int s = 0; s < 3; s++)
		for (int i = 0; i < 81; i++) {
			U.mutable_data()[s * 81 + i] = p.matrices.m[s].U[i];
			U1.mutable_data()[s * 81 + i] = p.matrices.m[s].U1[i];
		}
	py::array_t<double> pde({nv, (ssize_t)9});
	std::copy(p.pde.begin(), p.pde.end(), pde.mutable_data());
	py::list stages;
	for (int s = 0; s < 3; s++) {
		const auto& st = p.stages[s];
		py::array_t<int> kind({nv, (ssize_t)6}), v({nv, (ssize_t)6, (ssize_t)4}),
		    slot({nv, (ssize_t)6, (ssize_t)4});
		py::array_t<double> lam({nv, (ssize_t)6, (ssize_t)4}), q({nv, (ssize_t)6, (ssize_t)3});
		for (ssize_t e = 0; e < nv * 6; e++) {
			const gsx_foot& f = st.feet[(size_t)e];
			kind.mutable_data()[e] = f.kind;
			for (int i = 0; i < 4; i++) {
				v.mutable_data()[e * 4 + i] = f.v[i];
				slot.mutable_data()[e * 4 + i] = f.slot[i];
				lam.mutable_data()[e * 4 + i] = f.lam[i];
			}
			for (int i = 0; i < 3; i++) q.mutable_data()[e * 3 + i] = f.q[i];
		}
		py::dict d;
		d["kind"] = kind; d["v"] = v; d["slot"] = slot; d["lam"] = lam; d["q"] = q;
		stages.append(d);
	}
	py::dict d;
	d["id"] = p.id;
	d["coords"] = coords; d["cells"] = cells; d["U"] = U; d["U1"] = U1; d["pde"] = pde;
	d["tau"] = tau; d["average_height"] = p.averageHeight;
	d["maximal_eigenvalue"] = p.maximalEigenvalue;
	d["border"] = p.borderIdx; d["inner"] = p.innerIdx; d["contact"] = p.contactIdx;
	d["global"] = p.mesh.global;
	d["grad_offsets"] = p.gradient.offsets; d["grad_neighbors"] = p.gradient.neighbors;
	d["grad_rows"] = p.gradient.rows; d["grad_weights"] = p.gradient.weights;
	d["grad_M"] = p.gradient.M; d["grad_det"] = p.gradient.det;
	d["stages"] = stages;
	py::list outer;
	for (int s = 0; s < 3; s++) outer.append(std::vector<int>(p.stages[s].outerCode.begin(), p.stages[s].outerCode.end()));
	d["outer_code"] = outer;
	const auto& b = p.border;
	py::dict bd;
	bd["type"] = b.type; bd["min_det"] = b.minDet; bd["nodes"] = b.nodes; bd["cond"] = b.cond;
	bd["normal"] = b.normal; bd["B"] = b.B; bd["S"] = b.S;
	bd["outer"] = std::vector<int>(b.outer.begin(), b.outer.end());
	d["border_plan"] = bd;
	return d;
}

/// GPU-free simplex set-up: the first body's plans at the top level, every body in
/// "bodies", the contacts in "contacts".
py::dict simplexPlans(const Task& task) {
	using namespace simplex;
	const HostPlans hp = buildHostPlans(task);
	py::dict d = simplexBodyDict(hp.bodies.at(0), hp.tau);
	py::list bodies;
	for (const auto& b : hp.bodies) bodies.append(simplexBodyDict(b, hp.tau));
	d["bodies"] = bodies;
	py::list contacts;
	for (const auto& c : hp.contacts) {
		py::dict cd;
		cd["a"] = c.a; cd["b"] = c.b;
		cd["nodes_a"] = c.nodesA; cd["nodes_b"] = c.nodesB;
		cd["normal"] = c.normal; cd["S"] = c.S;
		cd["code_a"] = std::vector<int>(c.codeA.begin(), c.codeA.end());
		cd["code_b"] = std::vector<int>(c.codeB.begin(), c.codeB.end());
		cd["min_det"] = std::vector<double>(&c.minDet[0][0], &c.minDet[0][0] + 6);
		contacts.append(cd);
	}
	d["contacts"] = contacts;
	return d;
}

struct PySimplexEngine {
	std::shared_ptr<simplex::Engine> e;
	py::array_t<double> pde(size_t body) const {
		const std::vector<double> v = e->pde(body);
		py::array_t<double> out({(ssize_t)(v.size() / 9), (ssize_t)9});
		std::copy(v.begin(), v.end(), out.mutable_data());
		return out;
	}
};

}  // namespace

PYBIND11_MODULE(_gcm_host, m) {
	m.doc() = "C++ host mirror of libgcm's cubic Engine/Task surface over the gcmx C-ABI";
	py::register_exception<Exception>(m, "GcmException");

	py::class_<Task>(m, "Task")
	    .def(py::init<>())
	    .def_property("dimensionality", [](Task& t) { return t.globalSettings.dimensionality; },
	                  [](Task& t, int d) { t.globalSettings.dimensionality = d; })
	    .def_property("courant", [](Task& t) { return t.globalSettings.CourantNumber; },
	                  [](Task& t, real c) { t.globalSettings.CourantNumber = c; })
	    .def_property("number_of_snaps", [](Task& t) { return t.globalSettings.numberOfSnaps; },
	                  [](Task& t, int n) { t.globalSettings.numberOfSnaps = n; })
	    .def_property("steps_per_snap", [](Task& t) { return t.globalSettings.stepsPerSnap; },
	                  [](Task& t, int n) { t.globalSettings.stepsPerSnap = n; })
	    .def_property("required_time", [](Task& t) { return t.globalSettings.requiredTime; },
	                  [](Task& t, real r) { t.globalSettings.requiredTime = r; })
	    .def_property("border_size", [](Task& t) { return t.cubicGrid.borderSize; },
	                  [](Task& t, int b) { t.cubicGrid.borderSize = b; })
	    .def_property("h", [](Task& t) { return t.cubicGrid.h; },
	                  [](Task& t, std::vector<real> h) { t.cubicGrid.h = h; })
	    .def("add_body",
	         [](Task& t, size_t id, std::vector<int> sizes, std::vector<int> start) {
		         t.bodies[id] = Task::Body();
		         t.cubicGrid.cubics[id] = {sizes, start};
	         })
	    .def("set_default_material",
	         [](Task& t, real rho, real lam, real mu, real tau0, int number) {
		         t.materialConditions.type = Task::MaterialCondition::Type::BY_AREAS;
		         t.materialConditions.byAreas.defaultMaterial =
		             std::make_shared<IsotropicMaterial>(rho, lam, mu, 0, 0, number, tau0);
	         },
	         py::arg("rho"), py::arg("lam"), py::arg("mu"), py::arg("tau0") = 0.0,
	         py::arg("number") = 0)
	    .def("add_material",
	         [](Task& t, py::tuple area, real rho, real lam, real mu, real tau0, int number) {
		         t.materialConditions.byAreas.materials.push_back(
		             {makeArea(area), std::make_shared<IsotropicMaterial>(rho, lam, mu, 0, 0, number, tau0)});
	         },
	         py::arg("area"), py::arg("rho"), py::arg("lam"), py::arg("mu"), py::arg("tau0") = 0.0,
	         py::arg("number") = 0)
	    .def("set_body_material",
	         [](Task& t, size_t id, real rho, real lam, real mu, real tau0) {
		         t.materialConditions.type = Task::MaterialCondition::Type::BY_BODIES;
		         t.materialConditions.byBodies.bodyMaterialMap[id] =
		             std::make_shared<IsotropicMaterial>(rho, lam, mu, 0, 0, 0, tau0);
	         },
	         py::arg("id"), py::arg("rho"), py::arg("lam"), py::arg("mu"), py::arg("tau0") = 0.0)
	    .def_property("output_directory", [](Task& t) { return t.globalSettings.outputDirectory; },
	                  [](Task& t, const std::string& d) { t.globalSettings.outputDirectory = d; })
	    .def("add_snapshotter",
	         [](Task& t, const std::string& name) {
		         if (name == "VTK") t.globalSettings.snapshottersId.push_back(Snapshotters::T::VTK);
		         else if (name == "SLICESNAP") t.globalSettings.snapshottersId.push_back(Snapshotters::T::SLICESNAP);
		         else if (name == "DETECTOR") t.globalSettings.snapshottersId.push_back(Snapshotters::T::DETECTOR);
		         else throw Exception("unknown snapshotter " + name);
	         })
	    .def("set_vtk_quantities",
	         [](Task& t, std::vector<std::string> qs) {
		         t.vtkSnapshotter.quantitiesToSnap.clear();
		         for (auto& q : qs) t.vtkSnapshotter.quantitiesToSnap.push_back(quantity(q));
	         })
	    .def("set_detector",
	         [](Task& t, std::vector<std::string> qs, py::tuple area, size_t gridId) {
		         t.detector.quantities.clear();
		         for (auto& q : qs) t.detector.quantities.push_back(quantity(q));
		         t.detector.area = makeArea(area);
		         t.detector.gridId = gridId;
	         })
	    .def_property("grid", [](Task& t) {
		                  return std::string(t.globalSettings.gridId == Grids::T::SIMPLEX ? "SIMPLEX" : "CUBIC");
	                  },
	                  [](Task& t, const std::string& g) {
		                  if (g == "SIMPLEX") t.globalSettings.gridId = Grids::T::SIMPLEX;
		                  else if (g == "CUBIC") t.globalSettings.gridId = Grids::T::CUBIC;
		                  else throw Exception("unknown grid " + g);
	                  })
	    .def_property("calculation_basis", [](Task& t) { return t.calculationBasis; },
	                  [](Task& t, std::vector<real> b) { t.calculationBasis = b; })
	    .def("set_simplex_box",
	         [](Task& t, std::array<int, 3> cells, std::vector<real> lo, std::vector<real> hi,
	            real jitter, uint64_t seed) {
		         if (lo.size() != 3 || hi.size() != 3) throw Exception("set_simplex_box: 3-D box");
		         t.simplexGrid.cells = cells;
		         t.simplexGrid.lo = {lo[0], lo[1], lo[2]};
		         t.simplexGrid.hi = {hi[0], hi[1], hi[2]};
		         t.simplexGrid.jitter = jitter;
		         t.simplexGrid.seed = seed;
	         },
	         py::arg("cells"), py::arg("lo"), py::arg("hi"), py::arg("jitter") = 0.0,
	         py::arg("seed") = 0)
	    .def("add_ode",
	         [](Task& t, size_t id, const std::string& name) {
		         if (!t.bodies.count(id)) throw Exception("add_ode: no such body");
		         if (name == "MAXWELL_VISCOSITY") t.bodies[id].odes.push_back(Odes::T::MAXWELL_VISCOSITY);
		         else if (name == "CONTINUAL_DAMAGE") t.bodies[id].odes.push_back(Odes::T::CONTINUAL_DAMAGE);
		         else if (name == "IDEAL_PLASTIC_FLOW") t.bodies[id].odes.push_back(Odes::T::IDEAL_PLASTIC_FLOW);
		         else throw Exception("unknown ODE type " + name);
	         })
	    .def("add_initial_vector",
	         [](Task& t, py::tuple area, std::vector<real> v) {
		         t.initialCondition.vectors.push_back({makeArea(area), v});
	         })
	    .def("add_initial_wave",
	         [](Task& t, py::tuple area, const std::string& w, int direction, const std::string& q, real value) {
		         t.initialCondition.waves.push_back({makeArea(area), wave(w), direction, quantity(q), value});
	         })
	    .def("add_initial_quantity",
	         [](Task& t, py::tuple area, const std::string& q, real value) {
		         t.initialCondition.quantities.push_back({makeArea(area), quantity(q), value});
	         })
	    .def("add_border_condition",
	         [](Task& t, size_t body, int direction, py::tuple area,
	            std::map<std::string, std::function<real(real)>> values) {
		         Task::CubicBorderCondition bc;
		         bc.direction = direction;
		         bc.area = makeArea(area);
		         for (auto& kv : values) bc.values[quantity(kv.first)] = kv.second;
		         t.cubicBorderConditions[body].push_back(bc);
	         })
	    .def("add_simplex_border_condition",
	         [](Task& t, py::tuple area, const std::string& type,
	            std::vector<std::function<real(real)>> values, bool useForMulticontactNodes) {
		         // Task::borderConditions (Task.hpp:204-213)
		         Task::BorderCondition bc;
		         bc.area = makeArea(area);
		         if (type == "FIXED_FORCE") bc.type = BorderConditions::T::FIXED_FORCE;
		         else if (type == "FIXED_VELOCITY") bc.type = BorderConditions::T::FIXED_VELOCITY;
		         else throw Exception("unknown border condition type " + type);
		         bc.values = std::move(values);
		         bc.useForMulticontactNodes = useForMulticontactNodes;
		         t.borderConditions.push_back(bc);
	         },
	         py::arg("area"), py::arg("type"), py::arg("values"),
	         py::arg("use_for_multicontact_nodes") = true)
	    .def("set_simplex_inm_mesh",
	         [](Task& t, const std::string& fileName) {
		         t.simplexGrid.mesher = Task::SimplexGrid::Mesher::INM_MESHER;
		         t.simplexGrid.fileName = fileName;
	         },
	         py::arg("file_name"), "INM_MESHER: points, cells and per-cell body ids from a file")
	    .def("set_simplex_domain",
	         [](Task& t, std::vector<std::array<real, 3>> points, std::vector<std::array<int, 3>> faces) {
		         t.simplexGrid.offPoints.assign(points.begin(), points.end());
		         t.simplexGrid.offFaces = std::move(faces);
	         },
	         py::arg("points"), py::arg("faces"),
	         "Domain surface (closed triangles): cells whose centroid is outside are empty space")
	    .def("set_simplex_domain_off",
	         [](Task& t, const std::string& fileName) {
		         simplex::readOff(fileName, t.simplexGrid.offPoints, t.simplexGrid.offFaces);
	         },
	         py::arg("file_name"))
	    .def("add_simplex_body_area",
	         [](Task& t, py::tuple area, size_t id) {
		         t.simplexGrid.bodyAreas.push_back({makeArea(area), id});
	         },
	         py::arg("area"), py::arg("body"))
	    .def("set_contact_condition",
	         [](Task& t, const std::string& type, py::object pair) {
		         ContactConditions::T c;
		         if (type == "ADHESION") c = ContactConditions::T::ADHESION;
		         else if (type == "SLIDE") c = ContactConditions::T::SLIDE;
		         else throw Exception("unknown contact condition " + type);
		         if (pair.is_none()) t.contactCondition.defaultCondition = c;
		         else t.contactCondition.gridToGridConditions[pair.cast<std::pair<size_t, size_t>>()] = c;
	         },
	         py::arg("type"), py::arg("pair") = py::none(),
	         "Task::contactCondition: the default, or the condition of one pair of bodies");

	m.def(
	    "host_state",
	    [](const Task& t, size_t id) {
		    const int D = t.globalSettings.dimensionality;
		    if (D == 1) return hostState<1>(t, id);
		    if (D == 2) return hostState<2>(t, id);
		    if (D == 3) return hostState<3>(t, id);
		    throw Exception("dimensionality must be 1, 2 or 3");
	    },
	    "GPU-free MaterialsCondition + InitialCondition set-up of one body", py::arg("task"),
	    py::arg("body_id"));

	m.def(
	    "write_vtk",
	    [](const Task& t, size_t id, const std::string& fileName, py::object pde) {
		    const int D = t.globalSettings.dimensionality;
		    if (D == 1) return writeVtkHost<1>(t, id, fileName, pde);
		    if (D == 2) return writeVtkHost<2>(t, id, fileName, pde);
		    if (D == 3) return writeVtkHost<3>(t, id, fileName, pde);
		    throw Exception("dimensionality must be 1, 2 or 3");
	    },
	    "GPU-free VtkSnapshotter file of one body (set-up layer, or `pde`)", py::arg("task"),
	    py::arg("body_id"), py::arg("file_name"), py::arg("pde") = py::none());

	m.def(
	    "write_simplex_vtk",
	    [](const Task& t, const std::string& fileName, py::object pde, size_t body) {
		    // GPU-free simplex VtkSnapshotter file of one body: the set-up layer or `pde`
		    const simplex::HostPlans hp = simplex::buildHostPlans(t);
		    const simplex::BodyPlans& b = hp.bodies.at(body);
		    std::vector<real> u = b.pde;
		    if (!pde.is_none()) {
			    auto a = pde.cast<py::array_t<double, py::array::c_style | py::array::forcecast>>();
			    if ((size_t)a.size() != u.size()) throw Exception("pde has the wrong size");
			    std::copy(a.data(), a.data() + a.size(), u.begin());
		    }
		    simplex::writeVtkSnapshot(fileName, b.mesh.v, b.mesh.cells, u.data(),
		                              t.materialConditions.byBodies.bodyMaterialMap.at(b.id)->materialNumber,
		                              t.vtkSnapshotter.quantitiesToSnap);
	    },
	    py::arg("task"), py::arg("file_name"), py::arg("pde") = py::none(), py::arg("body") = 0);

	m.def(
	    "read_inm",
	    [](const std::string& fileName) {
		    std::vector<Real3> pts;
		    std::vector<std::array<int, 4>> cells;
		    std::vector<int> mats;
		    simplex::readInm(fileName, pts, cells, mats);
		    py::array_t<double> P({(ssize_t)pts.size(), (ssize_t)3});
		    for (size_t i = 0; i < pts.size(); i++)
			    for (int c = 0; c < 3; c++) P.mutable_at((ssize_t)i, c) = pts[i][c];
		    return py::make_tuple(P, cells, mats);
	    },
	    "InmMeshLoader::readFromFile: (points, cells (1-based), materials)", py::arg("file_name"));

	m.def(
	    "simplex_triangulation",
	    [](const Task& t) {
		    const simplex::Triangulation tr = simplex::buildTriangulation(t);
		    py::array_t<double> P({(ssize_t)tr.all.v.size(), (ssize_t)3});
		    for (size_t i = 0; i < tr.all.v.size(); i++)
			    for (int c = 0; c < 3; c++) P.mutable_at((ssize_t)i, c) = tr.all.v[i][c];
		    return py::make_tuple(P, tr.all.cells, tr.gridId);
	    },
	    "The task's whole triangulation: (points, cells (0-based), grid id per cell, -1 = empty)",
	    py::arg("task"));

	m.def(
	    "tet_barycentric",
	    [](const Real3& a, const Real3& b, const Real3& c, const Real3& d, const Real3& q) {
		    return simplex::barycentricCoordinates(a, b, c, d, q);
	    },
	    "linal::barycentricCoordinates of a tetrahedron (the stage plans' CELL-foot weights)");

	m.def(
	    "tet_owner_pick",
	    [](const std::array<Real3, 6>& pts, const Real3& q) {
		    Real3 p6[6];
		    for (int i = 0; i < 6; i++) p6[i] = pts[i];
		    int slot[4];
		    real lam[4];
		    simplex::interpolateInOwnerPick(p6, q, slot, lam);
		    return py::make_tuple(std::array<int, 4>{slot[0], slot[1], slot[2], slot[3]},
		                          std::array<real, 4>{lam[0], lam[1], lam[2], lam[3]});
	    },
	    "TetrahedronInterpolator::interpolateInOwner's choice as the stage plans make it: "
	    "(point indices, barycentrics); raises when no tetrahedron holds q",
	    py::arg("points"), py::arg("q"));

	m.def(
	    "gsl_lu",
	    [](py::array_t<double, py::array::c_style | py::array::forcecast> A, py::object b) {
		    // csrc/contact.hpp's restatement of gsl_linalg_LU_decomp / _det / _solve
		    // (GslUtils.hpp:96-168), the code the contact-corrector kernels run
		    if (A.ndim() != 2 || A.shape(0) != A.shape(1)) throw Exception("square matrix expected");
		    const int n = (int)A.shape(0);
		    auto run = [&](auto NC) -> py::object {
			    constexpr int N = decltype(NC)::value;
			    double LU[N][N], bb[N], x[N];
			    int perm[N], signum;
			    for (int i = 0; i < N; i++)
				    for (int j = 0; j < N; j++) LU[i][j] = A.at(i, j);
			    gsx::luDecomp<N>(LU, perm, signum);
			    const double det = gsx::luDet<N>(LU, signum);
			    if (b.is_none()) return py::float_(det);
			    auto bv = b.cast<std::vector<double>>();
			    if ((int)bv.size() != N) throw Exception("right-hand side of the wrong size");
			    // gsl_linalg_LU_solve: "matrix is singular" (solveLinearSystem throws)
			    if (gsx::luSingular<N>(LU)) throw Exception("gsl_linalg_LU_solve: matrix is singular");
			    for (int i = 0; i < N; i++) bb[i] = bv[i];
			    gsx::luSolve<N>(LU, perm, bb, x);
			    return py::cast(std::vector<double>(x, x + N));
		    };
		    switch (n) {
		    case 1: return run(std::integral_constant<int, 1>{});
		    case 2: return run(std::integral_constant<int, 2>{});
		    case 3: return run(std::integral_constant<int, 3>{});
		    case 4: return run(std::integral_constant<int, 4>{});
		    case 5: return run(std::integral_constant<int, 5>{});
		    case 6: return run(std::integral_constant<int, 6>{});
		    case 7: return run(std::integral_constant<int, 7>{});
		    case 8: return run(std::integral_constant<int, 8>{});
		    case 9: return run(std::integral_constant<int, 9>{});
		    default: throw Exception("1..9 rows supported");
		    }
	    },
	    "determinant (b None) or solution of A x = b through csrc/contact.hpp's GSL LU restatement",
	    py::arg("A"), py::arg("b") = py::none());

	m.def("simplex_plans", &simplexPlans,
	      "GPU-free simplex set-up: mesh, time step, gradient and stage plans", py::arg("task"));

	py::class_<PySimplexEngine>(m, "SimplexEngine")
	    .def(py::init([](const Task& t, int device) {
		         PySimplexEngine p;
		         p.e = std::make_shared<simplex::Engine>(t, device);
		         return p;
	         }),
	         py::arg("task"), py::arg("device") = 0)
	    // both end with a device check: a one-launch stage whose wait gave up
	    // (gsx_sync: GCMX_ERR_STATE) raises here instead of returning stale results
	    .def("run", [](PySimplexEngine& p) { p.e->run(); p.e->sync(); })
	    .def("run_steps", [](PySimplexEngine& p, int n, bool check) {
		         p.e->runSteps(n);
		         if (check) p.e->sync();
	         }, py::arg("n"), py::arg("check") = true)
	    .def("stage_plan_info", [](PySimplexEngine& p, size_t body, int stage) { return p.e->stagePlanInfo(body, stage); },
	         "(the plan admits the one-launch stage, inner feet that wait there)", py::arg("body"), py::arg("stage"))
	    .def("set_wait_budget", [](PySimplexEngine& p, int polls) { p.e->setWaitBudget(polls); },
	         "polls per device wait of the one-launch stages; < 0: every wait reports a timeout (tests)",
	         py::arg("polls"))
	    .def("pde", &PySimplexEngine::pde, "current layer of a body [n_vertices, 9]",
	         py::arg("body") = 0)
	    .def_property_readonly("number_of_bodies", [](PySimplexEngine& p) { return p.e->numberOfBodies(); })
	    .def_property_readonly("number_of_contact_pairs",
	                           [](PySimplexEngine& p) { return p.e->numberOfContactPairs(); })
	    .def("number_of_vertices", [](PySimplexEngine& p, size_t body) { return p.e->mesh(body).nVertices(); },
	         py::arg("body") = 0)
	    .def("sync", [](PySimplexEngine& p) { p.e->sync(); }, "wait for the bodies' streams")
	    .def("set_replay_steps", [](PySimplexEngine& p, bool on) { p.e->setReplaySteps(on); },
	         "gsx_step graph replay or the individual stage calls (default)", py::arg("on"))
	    .def("set_node_lanes", [](PySimplexEngine& p, int lanes) { p.e->setNodeLanes(lanes); },
	         "node-kernel layout: 0 automatic, 1 thread per node, 8 lanes per node", py::arg("lanes"))
	    .def("set_stage_fusion", [](PySimplexEngine& p, int mode) { p.e->setStageFusion(mode); },
	         "one launch per stage for a body without contacts: 0 off, 1 border + inner, "
	         "2 with the gradient, -1 (default) measured per mesh on the first steps", py::arg("mode"))
	    .def_property_readonly("stage_fusion", [](PySimplexEngine& p) { return p.e->stageFusion(); })
	    .def_property_readonly("fusion_tuning", [](PySimplexEngine& p) { return p.e->fusionTuning(); })
	    .def_property_readonly("fusion_times_ms", [](PySimplexEngine& p) { return p.e->fusionTimes(); })
	    .def_property_readonly("launches", [](PySimplexEngine& p) { return p.e->launches(); })
	    .def_property_readonly("fused_stages", [](PySimplexEngine& p) { return p.e->fusedStages(); })
	    .def_property_readonly("steps", [](PySimplexEngine& p) { return p.e->stepsDone(); })
	    .def_property_readonly("time_step", [](PySimplexEngine& p) { return p.e->timeStepValue(); })
	    .def_property_readonly("required_time", [](PySimplexEngine& p) { return p.e->getRequiredTime(); });

	py::class_<PyEngine>(m, "Engine")
	    .def(py::init([](const Task& t, int device) {
		         PyEngine p;
		         p.e = createEngine(t, device);
		         p.D = t.globalSettings.dimensionality;
		         return p;
	         }),
	         py::arg("task"), py::arg("device") = 0)
	    .def("run", [](PyEngine& p) { p.e->run(); })
	    .def("run_steps", &PyEngine::runSteps)
	    .def("pde", &PyEngine::pde, "current layer of a body, all nodes incl. ghosts [..., M]")
	    .def("path", &PyEngine::path)
	    .def("last_path", &PyEngine::lastPath)
	    .def("ode_fused", &PyEngine::odeFused)
	    .def("sync", &PyEngine::sync, py::arg("body") = 0)
	    .def("maximal_eigenvalue", &PyEngine::maximalEigenvalue)
	    .def_property_readonly("steps", [](PyEngine& p) { return p.e->stepsDone(); })
	    .def_property_readonly("required_time", [](PyEngine& p) { return p.e->getRequiredTime(); })
	    .def_property_readonly("time", [](PyEngine&) { return Clock::Time(); })
	    .def_property_readonly("time_step", [](PyEngine&) { return Clock::TimeStep(); });
}
