// task.hpp -- the subset of gcm::Task the cubic path reads, with the
// reference's field names (util/task/Task.hpp:24-234), plus areas
// (util/math/Area.hpp) and the physical-quantity getters/setters of
// VelocitySigmaVariables (rheology/variables/VelocitySigmaVariables.{hpp,cpp}).
#pragma once

#include <cmath>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <cstdint>
#include <string>
#include <vector>

#include "elastic_model.hpp"

namespace gcm {

using Real3 = std::array<real, 3>;

/// gcm::Exception analogue: every reference assert_* / THROW_* throws.
struct Exception : std::runtime_error {
	using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ enums --
// util/Enum.hpp:27-120 (same enumerator order: std::map iteration order of
// Task::CubicBorderCondition::values follows it).
struct PhysicalQuantities {
	enum class T {
		VELOCITY, FORCE, Vx, Vy, Vz, Sxx, Sxy, Sxz, Syy, Syz, Szz, RHO, PRESSURE, DAMAGE_MEASURE
	};
};
struct Waves {
	enum class T { P_FORWARD, P_BACKWARD, S1_FORWARD, S1_BACKWARD, S2_FORWARD, S2_BACKWARD };
};
struct Materials {
	enum class T { ISOTROPIC, ORTHOTROPIC };
};
struct Models {
	enum class T { ELASTIC, ACOUSTIC };
};
/// util/Enum.hpp:136-147
struct Snapshotters {
	enum class T { VTK, DETECTOR, SLICESNAP };
};
/// util/Enum.hpp:153-163
struct Odes {
	enum class T { MAXWELL_VISCOSITY, CONTINUAL_DAMAGE, IDEAL_PLASTIC_FLOW };
};
/// util/Enum.hpp: BorderConditions::T (simplex border correctors)
struct BorderConditions {
	enum class T { FIXED_FORCE, FIXED_VELOCITY };
};
struct Grids {
	enum class T { CUBIC, SIMPLEX };
};
/// util/Enum.hpp:70-76
struct ContactConditions {
	enum class T { ADHESION, SLIDE };
};

// ------------------------------------------------------------------ areas --
/// util/math/Area.hpp:8-120.  contains() is strict (points on the border are outside).
struct Area {
	virtual ~Area() = default;
	virtual bool contains(const Real3& c) const = 0;
};
struct InfiniteArea : Area {
	bool contains(const Real3&) const override { return true; }
};
struct AxisAlignedBoxArea : Area {
	Real3 min, max;
	AxisAlignedBoxArea(const Real3& mn, const Real3& mx) : min(mn), max(mx) {
		for (int i = 0; i < 3; i++)
			if (!((max[i] - min[i]) > 0.0)) throw Exception("AxisAlignedBoxArea: max must exceed min");
	}
	bool contains(const Real3& c) const override {
		for (int i = 0; i < 3; i++)
			if (c[i] <= min[i] || c[i] >= max[i]) return false;
		return true;
	}
};
struct SphereArea : Area {
	real radius;
	Real3 center;
	SphereArea(real r, const Real3& c) : radius(r), center(c) {
		if (!(radius > 0.0)) throw Exception("SphereArea: radius must be > 0");
	}
	bool contains(const Real3& c) const override {
		const real dx = c[0] - center[0], dy = c[1] - center[1], dz = c[2] - center[2];
		return std::sqrt(dx * dx + dy * dy + dz * dz) < radius;  // linal::length
	}
};
struct StraightBoundedCylinderArea : Area {
	real radius;
	Real3 begin, end, axis;
	StraightBoundedCylinderArea(real r, const Real3& b, const Real3& e) : radius(r), begin(b), end(e) {
		const Real3 d = {e[0] - b[0], e[1] - b[1], e[2] - b[2]};
		const real l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
		for (int i = 0; i < 3; i++) axis[i] = d[i] / l;
		if (!(radius > 0.0)) throw Exception("cylinder radius must be > 0");
	}
	bool contains(const Real3& c) const override {
		auto dot = [](const Real3& a, const Real3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
		const Real3 cb = {c[0] - begin[0], c[1] - begin[1], c[2] - begin[2]};
		const Real3 ce = {c[0] - end[0], c[1] - end[1], c[2] - end[2]};
		if (dot(cb, axis) * dot(ce, axis) >= 0) return false;
		const real p = dot(cb, axis);
		return dot(cb, cb) - p * p < radius * radius;
	}
};

// ------------------------------------------------- quantities on vectors --
/// Component of a scalar quantity in the D-dimensional velocity/sigma vector,
/// or -1 (VelocitySigmaVariables.cpp:22-66).
inline int quantityComponent(int D, PhysicalQuantities::T q) {
	using Q = PhysicalQuantities::T;
	switch (q) {
	case Q::Vx: return 0;
	case Q::Vy: return D > 1 ? 1 : -1;
	case Q::Vz: return D > 2 ? 2 : -1;
	case Q::Sxx: return detail::sigmaIndex(D, 0, 0);
	case Q::Sxy: return D > 1 ? detail::sigmaIndex(D, 0, 1) : -1;
	case Q::Sxz: return D > 2 ? detail::sigmaIndex(D, 0, 2) : -1;
	case Q::Syy: return D > 1 ? detail::sigmaIndex(D, 1, 1) : -1;
	case Q::Syz: return D > 2 ? detail::sigmaIndex(D, 1, 2) : -1;
	case Q::Szz: return D > 2 ? detail::sigmaIndex(D, 2, 2) : -1;
	default: return -1;
	}
}
inline bool hasQuantity(int D, PhysicalQuantities::T q) {
	return q == PhysicalQuantities::T::PRESSURE || quantityComponent(D, q) >= 0;
}
/// GetSetter::Get (getPressure = -trace / D, VelocitySigmaVariables.hpp:98-104)
inline real getQuantity(int D, PhysicalQuantities::T q, const real* v) {
	if (q == PhysicalQuantities::T::PRESSURE) {
		real trace = 0;
		for (int i = 0; i < D; i++) trace += v[detail::sigmaIndex(D, i, i)];
		return -trace / D;
	}
	const int c = quantityComponent(D, q);
	if (c < 0) throw Exception("quantity not present in the PDE vector");
	return v[c];
}
/// GetSetter::Set (setPressure clears the whole vector first, hpp:106-111)
inline void setQuantity(int D, PhysicalQuantities::T q, real value, real* v) {
	if (q == PhysicalQuantities::T::PRESSURE) {
		for (int i = 0; i < pdeSize(D); i++) v[i] = 0;
		for (int i = 0; i < D; i++) v[detail::sigmaIndex(D, i, i)] = -value;
		return;
	}
	const int c = quantityComponent(D, q);
	if (c < 0) throw Exception("quantity not present in the PDE vector");
	v[c] = value;
}
/// Column of U1 a wave type selects for isotropic media (Model.cpp:33-82).
inline int waveColumn(int D, Waves::T w) {
	const int col = static_cast<int>(w);
	if (col >= 2 * D) throw Exception("wave type not present in this dimensionality");
	return col;
}

// ------------------------------------------------------------------- task --
struct Task {
	typedef std::function<real(real)> TimeDependency;

	struct Body {
		Materials::T materialId = Materials::T::ISOTROPIC;
		Models::T modelId = Models::T::ELASTIC;
		std::vector<Odes::T> odes;  // only MAXWELL_VISCOSITY on this path (Ode.hpp:28-37)
	};
	std::map<size_t, Body> bodies;

	struct GlobalSettings {
		int dimensionality = 0;
		Grids::T gridId = Grids::T::CUBIC;
		real CourantNumber = 0;
		int numberOfSnaps = 0;
		int stepsPerSnap = 1;
		real requiredTime = 0;
		bool verboseTimeSteps = false;
		std::vector<Snapshotters::T> snapshottersId;
		std::string outputDirectory = "";
	} globalSettings;

	struct CubicGrid {
		struct Cube {
			std::vector<int> sizes;
			std::vector<int> start;
		};
		std::vector<real> h;
		int borderSize = 0;
		std::map<size_t, Cube> cubics;
	} cubicGrid;

	struct MaterialCondition {
		typedef std::shared_ptr<IsotropicMaterial> Material;
		enum class Type { BY_AREAS, BY_BODIES } type = Type::BY_AREAS;
		struct ByAreas {
			Material defaultMaterial;
			struct Inhomogenity {
				std::shared_ptr<Area> area;
				Material material;
			};
			std::vector<Inhomogenity> materials;
		} byAreas;
		struct ByBodies {
			std::map<size_t, Material> bodyMaterialMap;
		} byBodies;
	} materialConditions;

	struct InitialCondition {
		struct Vector {
			std::shared_ptr<Area> area;
			std::vector<real> list;
		};
		std::vector<Vector> vectors;
		struct Wave {
			std::shared_ptr<Area> area;
			Waves::T waveType;
			int direction;
			PhysicalQuantities::T quantity;
			real quantityValue;
		};
		std::vector<Wave> waves;
		struct Quantity {
			std::shared_ptr<Area> area;
			PhysicalQuantities::T physicalQuantity;
			real value;
		};
		std::vector<Quantity> quantities;
	} initialCondition;

	struct CubicBorderCondition {
		int direction;
		std::shared_ptr<Area> area;
		typedef std::map<PhysicalQuantities::T, TimeDependency> Values;
		Values values;
	};
	std::map<size_t, std::vector<CubicBorderCondition>> cubicBorderConditions;

	/// Task::BorderCondition (Task.hpp:204-213): simplex border correctors.
	/// `values` are the OUTER_NUMBER = 3 components of b(t) in the border's
	/// local basis (util/task/BorderCondition.hpp).
	struct BorderCondition {
		std::shared_ptr<Area> area;
		bool useForMulticontactNodes = true;
		BorderConditions::T type = BorderConditions::T::FIXED_FORCE;
		std::vector<TimeDependency> values;
	};
	std::vector<BorderCondition> borderConditions;

	/// Task::ContactCondition (Task.hpp:216-220): simplex contact correctors between
	/// bodies (pair key = (smaller id, larger id)).
	struct ContactCondition {
		ContactConditions::T defaultCondition = ContactConditions::T::ADHESION;
		std::map<std::pair<size_t, size_t>, ContactConditions::T> gridToGridConditions;
	} contactCondition;

	/// The reference's Task::calculationBasis (Task.hpp:129): 9 numbers, column i =
	/// direction of stage i.  Required (constant) on the simplex path here.
	std::vector<real> calculationBasis;

	/// Task::SimplexGrid (Task.hpp:84-127) -- CGAL is absent, so the mesh is the
	/// jittered Kuhn tetrahedralisation of a box (simplex::boxMesh).
	struct SimplexGrid {
		/// Task::SimplexGrid::Mesher (Task.hpp:86-90): BOX_MESHER (this build's
		/// stand-in for CGAL_MESHER, absent) or INM_MESHER (fileName: points,
		/// cells and per-cell grid ids, InmMeshLoader.hpp)
		enum class Mesher { BOX_MESHER, INM_MESHER } mesher = Mesher::BOX_MESHER;
		std::string fileName;
		std::array<int, 3> cells = {0, 0, 0};  // cubes per axis
		Real3 lo = {0, 0, 0}, hi = {1, 1, 1};
		real jitter = 0;
		uint64_t seed = 0;
		/// Domain surface (the triangles of an .off file, Task.hpp:95 fileName):
		/// cells whose centroid is outside it (odd crossing parity -> inside, so
		/// inner closed surfaces such as layers_with_fracture.off's fracture are
		/// cavities) belong to the empty space.  Empty = the whole box.
		std::vector<Real3> offPoints;
		std::vector<std::array<int, 3>> offFaces;
		/// Cell -> body: the last rule whose area contains the cell centroid picks
		/// the body id, the first body otherwise (per-cell grid ids, as the INM
		/// mesher assigns them, InmMeshLoader.hpp:58-78).
		std::vector<std::pair<std::shared_ptr<Area>, size_t>> bodyAreas;
	} simplexGrid;

	struct VtkSnapshotter {
		/// list of physical quantities to write to vtk
		std::vector<PhysicalQuantities::T> quantitiesToSnap;
	} vtkSnapshotter;

	struct Detector {
		std::vector<PhysicalQuantities::T> quantities;
		std::shared_ptr<Area> area;
		size_t gridId = 0;
	} detector;
};

}  // namespace gcm
