// snapshot.cpp -- file writers of the snapshotters (see snapshot.hpp).
#include "snapshot.hpp"

#include <sys/stat.h>

#include <cerrno>
#include <cstdint>
#include <fstream>
#include <iomanip>
#include <sstream>

namespace gcm {

std::string zeroPadded(int number, int length) {
	std::ostringstream s;
	s << std::setfill('0') << std::setw(length) << number;
	return s.str();
}

void writeColumns(const std::string& fileName, const std::vector<std::vector<real>>& cols) {
	if (cols.empty()) throw Exception("writeColumns: no columns");
	for (const auto& c : cols)
		if (c.size() != cols[0].size()) throw Exception("writeColumns: ragged columns");
	std::ofstream f(fileName, std::ios::out);
	if (!f.is_open()) throw Exception("cannot open " + fileName);
	for (size_t i = 0; i < cols[0].size(); i++) {
		for (const auto& c : cols) f << c[i] << "\t";
		f << std::endl;
	}
}

void makeParentDirectories(const std::string& fileName) {
	for (size_t p = fileName.find('/'); p != std::string::npos; p = fileName.find('/', p + 1)) {
		if (p == 0) continue;
		const std::string dir = fileName.substr(0, p);
		if (mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST)
			throw Exception("cannot create directory " + dir);
	}
}

std::string Snapshotter::makeFileNameForSnapshot(const std::string& meshId, const int step,
                                                 const std::string& fileExtension,
                                                 const std::string& folder) const {
	const std::string mesh = "mesh" + meshId;
	const std::string snap = (step >= 0) ? "snap" + zeroPadded(step, 4) : "";
	const std::string core = "core" + zeroPadded(0, 2);
	std::string snapsDir = "snapshots";
	if (!outDir.empty()) snapsDir += "/" + outDir;
	const std::string name = snapsDir + "/" + folder + "/" + mesh + core + snap + "." + fileExtension;
	makeParentDirectories(name);
	return name;
}

namespace cubic {
const char* quantityName(PhysicalQuantities::T q);
}

namespace simplex {

void writeVtu(const std::string& fileName, const std::vector<float>& points,
              const std::vector<std::array<int, 4>>& cells, const std::vector<VtkPointArray>& arrays) {
	const uint64_t n = points.size() / 3, nc = cells.size();
	if (points.size() != 3 * n) throw Exception("writeVtu: points size");
	for (const auto& a : arrays)
		if (a.values.size() != n * (uint64_t)a.components) throw Exception("writeVtu: array size");
	std::vector<int64_t> conn, offs;
	std::vector<uint8_t> types(nc, 10);  // VTK_TETRA
	for (const auto& c : cells) {
		for (int x : c) {
			if (x < 0 || (uint64_t)x >= n) throw Exception("writeVtu: cell vertex out of range");
			conn.push_back(x);
		}
		offs.push_back((int64_t)conn.size());
	}
	std::ofstream f(fileName, std::ios::binary);
	if (!f.is_open()) throw Exception("cannot open " + fileName);
	f << "<?xml version=\"1.0\"?>\n"
	  << "<VTKFile type=\"UnstructuredGrid\" version=\"1.0\" byte_order=\"LittleEndian\" "
	     "header_type=\"UInt64\">\n"
	  << "  <UnstructuredGrid>\n"
	  << "    <Piece NumberOfPoints=\"" << n << "\" NumberOfCells=\"" << nc << "\">\n"
	  << "      <PointData>\n";
	uint64_t offset = 0;
	for (const auto& a : arrays) {
		f << "        <DataArray type=\"Float32\" Name=\"" << a.name << "\" NumberOfComponents=\""
		  << a.components << "\" format=\"appended\" offset=\"" << offset << "\"/>\n";
		offset += 8 + 4 * (uint64_t)a.values.size();
	}
	f << "      </PointData>\n      <CellData>\n      </CellData>\n      <Points>\n"
	  << "        <DataArray type=\"Float32\" Name=\"Points\" NumberOfComponents=\"3\" "
	     "format=\"appended\" offset=\"" << offset << "\"/>\n      </Points>\n      <Cells>\n";
	offset += 8 + 4 * (uint64_t)points.size();
	f << "        <DataArray type=\"Int64\" Name=\"connectivity\" format=\"appended\" offset=\""
	  << offset << "\"/>\n";
	offset += 8 + 8 * (uint64_t)conn.size();
	f << "        <DataArray type=\"Int64\" Name=\"offsets\" format=\"appended\" offset=\"" << offset
	  << "\"/>\n";
	offset += 8 + 8 * (uint64_t)offs.size();
	f << "        <DataArray type=\"UInt8\" Name=\"types\" format=\"appended\" offset=\"" << offset
	  << "\"/>\n      </Cells>\n    </Piece>\n  </UnstructuredGrid>\n"
	  << "  <AppendedData encoding=\"raw\">\n   _";
	auto block = [&f](const void* data, uint64_t bytes) {
		f.write(reinterpret_cast<const char*>(&bytes), 8);
		f.write(reinterpret_cast<const char*>(data), (std::streamsize)bytes);
	};
	for (const auto& a : arrays) block(a.values.data(), 4 * (uint64_t)a.values.size());
	block(points.data(), 4 * (uint64_t)points.size());
	block(conn.data(), 8 * (uint64_t)conn.size());
	block(offs.data(), 8 * (uint64_t)offs.size());
	block(types.data(), (uint64_t)types.size());
	f << "\n  </AppendedData>\n</VTKFile>\n";
	if (!f.good()) throw Exception("write failed: " + fileName);
}

void writeVtkSnapshot(const std::string& fileName, const std::vector<Real3>& coords,
                      const std::vector<std::array<int, 4>>& cells, const real* pde,
                      int materialNumber, const std::vector<PhysicalQuantities::T>& quantities) {
	const size_t n = coords.size();
	std::vector<float> points(3 * n);
	VtkPointArray vel{"Velocity", 3, std::vector<float>(3 * n)};
	std::vector<VtkPointArray> qs;
	for (auto q : quantities) {
		if (!hasQuantity(3, q)) throw Exception("quantity to snap is not in this PDE vector");
		qs.push_back(VtkPointArray{cubic::quantityName(q), 1, std::vector<float>(n)});
	}
	VtkPointArray mat{"material_index", 1, std::vector<float>(n, (float)materialNumber)};
	for (size_t p = 0; p < n; p++) {  // VtkIterator: vertices in local order
		const real* v = pde + 9 * p;
		for (int i = 0; i < 3; i++) {
			points[3 * p + i] = (float)coords[p][i];
			vel.values[3 * p + i] = (float)v[i];
		}
		for (size_t k = 0; k < qs.size(); k++) qs[k].values[p] = (float)getQuantity(3, quantities[k], v);
	}
	std::vector<VtkPointArray> arrays;
	arrays.push_back(std::move(vel));
	for (auto& a : qs) arrays.push_back(std::move(a));
	arrays.push_back(std::move(mat));
	writeVtu(fileName, points, cells, arrays);
}

}  // namespace simplex

namespace cubic {

const char* quantityName(PhysicalQuantities::T q) {  // util/Enum.cpp:5-21
	typedef PhysicalQuantities::T Q;
	switch (q) {
	case Q::VELOCITY: return "Velocity";
	case Q::FORCE: return "Force";
	case Q::Vx: return "Vx";
	case Q::Vy: return "Vy";
	case Q::Vz: return "Vz";
	case Q::Sxx: return "Sxx";
	case Q::Sxy: return "Sxy";
	case Q::Sxz: return "Sxz";
	case Q::Syy: return "Syy";
	case Q::Syz: return "Syz";
	case Q::Szz: return "Szz";
	case Q::RHO: return "rho";
	case Q::PRESSURE: return "pressure";
	case Q::DAMAGE_MEASURE: return "damage_measure";
	}
	return "unknown";
}

void writeVts(const std::string& fileName, const int dims[3], const std::vector<float>& points,
              const std::vector<VtsArray>& arrays) {
	const uint64_t n = (uint64_t)dims[0] * dims[1] * dims[2];
	if (points.size() != 3 * n) throw Exception("writeVts: points size");
	for (const auto& a : arrays)
		if (a.values.size() != n * (uint64_t)a.components) throw Exception("writeVts: array size");
	std::ofstream f(fileName, std::ios::binary);
	if (!f.is_open()) throw Exception("cannot open " + fileName);
	std::ostringstream ext;
	ext << "0 " << dims[0] - 1 << " 0 " << dims[1] - 1 << " 0 " << dims[2] - 1;
	f << "<?xml version=\"1.0\"?>\n"
	  << "<VTKFile type=\"StructuredGrid\" version=\"1.0\" byte_order=\"LittleEndian\" "
	     "header_type=\"UInt64\">\n"
	  << "  <StructuredGrid WholeExtent=\"" << ext.str() << "\">\n"
	  << "    <Piece Extent=\"" << ext.str() << "\">\n"
	  << "      <PointData>\n";
	uint64_t offset = 0;
	for (const auto& a : arrays) {
		f << "        <DataArray type=\"Float32\" Name=\"" << a.name << "\" NumberOfComponents=\""
		  << a.components << "\" format=\"appended\" offset=\"" << offset << "\"/>\n";
		offset += 8 + 4 * (uint64_t)a.values.size();
	}
	f << "      </PointData>\n      <CellData>\n      </CellData>\n      <Points>\n"
	  << "        <DataArray type=\"Float32\" Name=\"Points\" NumberOfComponents=\"3\" "
	     "format=\"appended\" offset=\""
	  << offset << "\"/>\n"
	  << "      </Points>\n    </Piece>\n  </StructuredGrid>\n"
	  << "  <AppendedData encoding=\"raw\">\n   _";
	auto block = [&f](const std::vector<float>& v) {
		const uint64_t bytes = 4 * (uint64_t)v.size();
		f.write(reinterpret_cast<const char*>(&bytes), 8);
		f.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)bytes);
	};
	for (const auto& a : arrays) block(a.values);
	block(points);
	f << "\n  </AppendedData>\n</VTKFile>\n";
	if (!f.good()) throw Exception("write failed: " + fileName);
}

template <int D>
void writeVtkSnapshot(const std::string& fileName, const std::array<int, D>& sizes,
                      const std::array<int, D>& start, const std::array<real, D>& h,
                      int borderSize, const real* pdeAll, const uint8_t* matIdAll,
                      const std::vector<int>& materialNumbers,
                      const std::vector<PhysicalQuantities::T>& quantities) {
	constexpr int M = pdeSize(D);
	int dims[3] = {1, 1, 1};
	for (int i = 0; i < D; i++) dims[i] = sizes[i];
	const size_t n = (size_t)dims[0] * dims[1] * dims[2];
	// CubicGrid indexMaker (CubicGrid.hpp:202-225): X slowest, last axis fastest
	long long im[3] = {0, 0, 0};
	const long long b2 = 2LL * borderSize;
	if (D == 1) im[0] = 1;
	if (D == 2) { im[0] = b2 + sizes[D - 1]; im[1] = 1; }
	if (D == 3) { im[0] = (b2 + sizes[1 % D]) * (b2 + sizes[D - 1]); im[1] = b2 + sizes[D - 1]; im[2] = 1; }
	std::vector<float> points(3 * n);
	VtsArray vel{"Velocity", 3, std::vector<float>(3 * n)};
	std::vector<VtsArray> qs;
	for (auto q : quantities) {
		if (!hasQuantity(D, q)) throw Exception("quantity to snap is not in this PDE vector");
		qs.push_back(VtsArray{quantityName(q), 1, std::vector<float>(n)});
	}
	VtsArray mat{"material_index", 1, std::vector<float>(n)};
	// SlowZFastX (VtkIterator, CubicGrid.hpp:34): x fastest
	size_t p = 0;
	for (int z = 0; z < dims[2]; z++)
		for (int y = 0; y < dims[1]; y++)
			for (int x = 0; x < dims[0]; x++, p++) {
				const int it[3] = {x, y, z};
				long long idx = 0;
				for (int i = 0; i < D; i++) idx += im[i] * (it[i] + borderSize);
				const real* v = pdeAll + (size_t)idx * M;
				for (int i = 0; i < 3; i++) {
					const real c = i < D ? (real)start[i] * h[i] + (real)it[i] * h[i] : 0;
					points[3 * p + i] = (float)c;
					vel.values[3 * p + i] = i < D ? (float)v[i] : 0.0f;  // getVelocity, padded
				}
				for (size_t k = 0; k < qs.size(); k++)
					qs[k].values[p] = (float)getQuantity(D, quantities[k], v);
				const int m = matIdAll ? matIdAll[idx] : 0;
				mat.values[p] = (float)materialNumbers.at((size_t)m);
			}
	std::vector<VtsArray> arrays;
	arrays.push_back(std::move(vel));
	for (auto& a : qs) arrays.push_back(std::move(a));
	arrays.push_back(std::move(mat));
	writeVts(fileName, dims, points, arrays);
}

template void writeVtkSnapshot<1>(const std::string&, const std::array<int, 1>&,
                                  const std::array<int, 1>&, const std::array<real, 1>&, int,
                                  const real*, const uint8_t*, const std::vector<int>&,
                                  const std::vector<PhysicalQuantities::T>&);
template void writeVtkSnapshot<2>(const std::string&, const std::array<int, 2>&,
                                  const std::array<int, 2>&, const std::array<real, 2>&, int,
                                  const real*, const uint8_t*, const std::vector<int>&,
                                  const std::vector<PhysicalQuantities::T>&);
template void writeVtkSnapshot<3>(const std::string&, const std::array<int, 3>&,
                                  const std::array<int, 3>&, const std::array<real, 3>&, int,
                                  const real*, const uint8_t*, const std::vector<int>&,
                                  const std::vector<PhysicalQuantities::T>&);

}  // namespace cubic
}  // namespace gcm
