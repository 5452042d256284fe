// snapshot.hpp -- snapshotters of the cubic engine (util/snapshot/*.hpp).
//
// These are the device -> host sync points of a run: a snapshot downloads the
// current layer once (HipMesh::pdeAll) and writes it on the host.
//   Snapshotter        (util/snapshot/Snapshotter.hpp:19-95)      -> gcm::Snapshotter
//   VtkSnapshotter     (util/snapshot/VtkSnapshotter.hpp:12-86)   -> cubic::VtkSnapshotter<D>
//   SliceSnapshotter   (util/snapshot/SliceSnapshotter.hpp:12-118)-> cubic::SliceSnapshotter<D>
// VTK itself is not in this image, so the VTK XML StructuredGrid (.vts) file is
// written directly (format of vtkXMLStructuredGridWriter: appended raw binary,
// UInt64 headers, Float32 arrays -- the reference's vtkFloatArray / vtkPoints).
#pragma once

#include <string>
#include <vector>

#include "task.hpp"

namespace gcm {

class AbstractGrid;

/// util/snapshot/Snapshotter.hpp:19-95
class Snapshotter {
public:
	typedef float precision;
	explicit Snapshotter(const Task& task)
	    : stepsPerSnap(task.globalSettings.stepsPerSnap),
	      outDir(task.globalSettings.outputDirectory) {}
	virtual ~Snapshotter() = default;
	/// Snapshotter.hpp:46-50
	void snapshot(const AbstractGrid* grid, const int step) {
		if (step % stepsPerSnap == 0) snapshotImpl(grid, step);
	}

protected:
	virtual void snapshotImpl(const AbstractGrid* grid, const int step) = 0;
	/// Snapshotter.hpp:56-77: snapshots[/outDir]/folder/mesh<id>core00snap<step>.<ext>
	/// (one process per body here: core = 00).  Creates the directories.
	std::string makeFileNameForSnapshot(const std::string& meshId, const int step,
	                                    const std::string& fileExtension,
	                                    const std::string& folder) const;

private:
	int stepsPerSnap = 1;
	std::string outDir;
};

/// FileUtils::writeStdVectorsToTextFile (util/FileUtils.hpp:25-31, 69-82): row i
/// = every column's i-th value followed by a tab, default stream formatting.
void writeColumns(const std::string& fileName, const std::vector<std::vector<real>>& cols);
/// util/StringUtils.hpp:15-19
std::string zeroPadded(int number, int length);
/// mkdir -p of the directory part of `fileName`
void makeParentDirectories(const std::string& fileName);

/// VtkSnapshotter's arrays of one vertex list (VtkSnapshotter.hpp:28-70):
/// "Velocity", the quantities by name, "material_index" -- name, components, values.
struct VtkPointArray {
	std::string name;
	int components = 1;
	std::vector<float> values;
};

namespace simplex {

/// Write a VTK XML UnstructuredGrid (.vtu) file of tetrahedra (what
/// vtkXMLUnstructuredGridWriter makes of VtkUtils' SimplexGrid output,
/// VtkUtils.hpp:54-66, 140-160): points (3 floats per vertex), cells (4 vertex
/// indices each, VTK_TETRA), the point arrays in order.  Appended raw binary.
void writeVtu(const std::string& fileName, const std::vector<float>& points,
              const std::vector<std::array<int, 4>>& cells, const std::vector<VtkPointArray>& arrays);

/// VtkSnapshotter::snapshotImpl (VtkSnapshotter.hpp:20-61) for a simplex body:
/// the vertex coordinates, pde [n][9], one material number for the body.  GPU-free.
void writeVtkSnapshot(const std::string& fileName, const std::vector<Real3>& coords,
                      const std::vector<std::array<int, 4>>& cells, const real* pde,
                      int materialNumber, const std::vector<PhysicalQuantities::T>& quantities);

/// The simplex VtkSnapshotter: file naming of Snapshotter (snapshots/vtk/mesh<id>
/// core00snap<step>.vtu) on top of writeVtkSnapshot.
class VtkSnapshotter : public Snapshotter {
public:
	explicit VtkSnapshotter(const Task& task)
	    : Snapshotter(task), quantities(task.vtkSnapshotter.quantitiesToSnap) {}
	std::string fileName(size_t meshId, int step) const {
		return makeFileNameForSnapshot(std::to_string(meshId), step, "vtu", "vtk");
	}
	const std::vector<PhysicalQuantities::T> quantities;

protected:
	void snapshotImpl(const AbstractGrid*, const int) override {
		throw Exception("simplex::VtkSnapshotter writes through simplex::Engine::writeSnapshots");
	}
};

}  // namespace simplex

namespace cubic {

/// One named Float32 point array of a .vts file (components 1 or 3).
struct VtsArray {
	std::string name;
	int components = 1;
	std::vector<float> values;  // VTK point order (x fastest), components interleaved
};

/// Write a VTK XML StructuredGrid file: `dims` points per axis (1 for axes >= D),
/// `points` 3 floats per point in VTK order, the point arrays in order.
void writeVts(const std::string& fileName, const int dims[3], const std::vector<float>& points,
              const std::vector<VtsArray>& arrays);

/// The arrays VtkSnapshotter::snapshotImpl writes (VtkSnapshotter.hpp:28-70) for a
/// layer in the reference AoS all-nodes order: "Velocity" (3 components, zero
/// padded), each quantity of `quantities` by its PhysicalQuantities::NAME, and
/// "material_index" (IsotropicMaterial::materialNumber of the node).  GPU-free.
template <int D>
void writeVtkSnapshot(const std::string& fileName, const std::array<int, D>& sizes,
                      const std::array<int, D>& start, const std::array<real, D>& h,
                      int borderSize, const real* pdeAll, const uint8_t* matIdAll,
                      const std::vector<int>& materialNumbers,
                      const std::vector<PhysicalQuantities::T>& quantities);

const char* quantityName(PhysicalQuantities::T q);

}  // namespace cubic
}  // namespace gcm
