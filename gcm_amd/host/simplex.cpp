// simplex.cpp -- mesh, triangulation queries and static plans of the simplex
// path (see simplex.hpp).  Every geometric predicate restates the reference's
// linal code operation by operation (paths relative to src/libgcm).
#include "simplex.hpp"

#include "../csrc/contact.hpp"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <map>
#include <sstream>
#include <memory>
#include <limits>
#include <set>

namespace gcm {
namespace simplex {

// ----------------------------------------------------------------- linal --
namespace {

inline Real3 sub(const Real3& a, const Real3& b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
inline Real3 add(const Real3& a, const Real3& b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2]}; }
inline Real3 mul(const Real3& a, real x) { return {a[0] * x, a[1] * x, a[2] * x}; }
inline real dot(const Real3& a, const Real3& b) {  // functions.hpp:327-334
	real r = a[0] * b[0];
	r += a[1] * b[1];
	r += a[2] * b[2];
	return r;
}
inline real length(const Real3& a) { return std::sqrt(dot(a, a)); }
inline Real3 cross(const Real3& a, const Real3& b) {  // geometry.hpp:13-17
	return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
inline Real3 normalize(const Real3& a) {
	const real l = length(a);
	return {a[0] / l, a[1] / l, a[2] / l};
}
/// determinants.hpp:40-53 (arbitrary-type 3x3) and :25-30 (2x2)
inline real det3(real m11, real m12, real m13, real m21, real m22, real m23, real m31, real m32,
                 real m33) {
	return m11 * (m22 * m33 - m23 * m32) - m12 * (m21 * m33 - m23 * m31) +
	       m13 * (m21 * m32 - m22 * m31);
}
inline real det2(real m11, real m12, real m21, real m22) { return m11 * m22 - m12 * m21; }
/// linearSystems.hpp:104-129 (Cramer); throws like THROW_INVALID_ARG
Real3 solve3(const real A[3][3], const Real3& b) {
	const real det = det3(A[0][0], A[0][1], A[0][2], A[1][0], A[1][1], A[1][2], A[2][0], A[2][1],
	                      A[2][2]);
	if (det == 0) throw Exception("SLE determinant is zero");
	const real d1 = det3(b[0], A[0][1], A[0][2], b[1], A[1][1], A[1][2], b[2], A[2][1], A[2][2]);
	const real d2 = det3(A[0][0], b[0], A[0][2], A[1][0], b[1], A[1][2], A[2][0], b[2], A[2][2]);
	const real d3 = det3(A[0][0], A[0][1], b[0], A[1][0], A[1][1], b[1], A[2][0], A[2][1], b[2]);
	return {d1 / det, d2 / det, d3 / det};
}
/// linearLeastSquares (linearSystems.hpp:150-158) for a 3x2 system, W = I:
/// solve(A^T (W A), A^T (W b)) with transposeMultiply's summation order.
std::array<real, 2> lls32(const Real3& c0, const Real3& c1, const Real3& b) {
	const Real3* col[2] = {&c0, &c1};
	real M[2][2], r[2];
	for (int i = 0; i < 2; i++) {
		for (int j = 0; j < 2; j++) {
			real s = (*col[i])[0] * (*col[j])[0];
			for (int n = 1; n < 3; n++) s += (*col[i])[n] * (*col[j])[n];
			M[i][j] = s;
		}
		real s = (*col[i])[0] * b[0];
		for (int n = 1; n < 3; n++) s += (*col[i])[n] * b[n];
		r[i] = s;
	}
	const real det = det2(M[0][0], M[0][1], M[1][0], M[1][1]);  // linearSystems.hpp:71-90
	if (det == 0) throw Exception("SLE determinant is zero");
	return {det2(r[0], M[0][1], r[1], M[1][1]) / det, det2(M[0][0], r[0], M[1][0], r[1]) / det};
}
/// 3x1 system (segment barycentrics): (A^T A)^-1 A^T b, 1x1 solve
real lls31(const Real3& c0, const Real3& b) {
	real m = c0[0] * c0[0];
	for (int n = 1; n < 3; n++) m += c0[n] * c0[n];
	real r = c0[0] * b[0];
	for (int n = 1; n < 3; n++) r += c0[n] * b[n];
	if (m == 0) throw Exception("SLE determinant is zero");
	return r / m;
}
/// geometry.hpp:142-151
std::array<real, 4> barycentric(const Real3& a, const Real3& b, const Real3& c, const Real3& d,
                                const Real3& q) {
	const real T[3][3] = {{a[0] - d[0], b[0] - d[0], c[0] - d[0]},
	                      {a[1] - d[1], b[1] - d[1], c[1] - d[1]},
	                      {a[2] - d[2], b[2] - d[2], c[2] - d[2]}};
	const Real3 l = solve3(T, sub(q, d));
	return {l[0], l[1], l[2], 1 - l[0] - l[1] - l[2]};
}
/// geometry.hpp:124-137 (triangle in 3-D)
Real3 barycentric3(const Real3& a, const Real3& b, const Real3& c, const Real3& q) {
	const auto l = lls32(sub(a, c), sub(b, c), sub(q, c));
	return {l[0], l[1], 1 - l[0] - l[1]};
}
/// geometry.hpp:88-103 (segment in 3-D)
std::array<real, 2> barycentric2(const Real3& a, const Real3& b, const Real3& q) {
	const real l = lls31(sub(a, b), sub(q, b));
	return {l, 1 - l};
}
/// geometry.hpp:248-261
real orientedVolume(const Real3& a, const Real3& b, const Real3& c, const Real3& d) {
	const Real3 ba = sub(b, a), ca = sub(c, a), da = sub(d, a);
	return det3(ba[0], ba[1], ba[2], ca[0], ca[1], ca[2], da[0], da[1], da[2]) / 6;
}
real volume(const Real3& a, const Real3& b, const Real3& c, const Real3& d) {
	return std::fabs(orientedVolume(a, b, c, d));
}
real area(const Real3& a, const Real3& b, const Real3& c) {  // geometry.hpp:238-240
	return length(cross(sub(b, a), sub(c, a))) / 2;
}
real minimalHeight3(const Real3& a, const Real3& b, const Real3& c) {  // geometry.hpp:263-270
	const real S = area(a, b, c);
	const real ab = length(sub(a, b)), ac = length(sub(a, c)), bc = length(sub(b, c));
	return 2 * S / std::fmax(ab, std::fmax(ac, bc));
}
real minimalHeight4(const Real3& a, const Real3& b, const Real3& c, const Real3& d) {  // :274-284
	const real V = volume(a, b, c, d);
	const real A = area(b, c, d), B = area(c, d, a), C = area(d, a, b), D = area(a, b, c);
	return 3 * V / std::fmax(A, std::fmax(B, std::fmax(C, D)));
}
bool isDegenerate3(const Real3& a, const Real3& b, const Real3& c, real eps) {  // :291-297
	const real h = minimalHeight3(a, b, c);
	const real l = (length(sub(a, b)) + length(sub(a, c)) + length(sub(b, c))) / 3;
	return h <= eps * l;
}
bool isDegenerate4(const Real3& a, const Real3& b, const Real3& c, const Real3& d, real eps) {
	const real h = minimalHeight4(a, b, c, d);  // :304-310
	const real l = (length(sub(a, b)) + length(sub(a, c)) + length(sub(a, d)) + length(sub(d, b)) +
	                length(sub(d, c)) + length(sub(b, c))) /
	               6;
	return h <= eps * l;
}
bool segmentContains(const Real3& a, const Real3& b, const Real3& q, real eps, real degEps) {
	if (!isDegenerate3(a, b, q, degEps)) return false;  // :338-343
	const auto l = barycentric2(a, b, q);
	return l[0] >= -eps && l[1] >= -eps;
}
bool triangleContains(const Real3& a, const Real3& b, const Real3& c, const Real3& q, real eps,
                      real degEps) {  // :359-364
	if (!isDegenerate4(a, b, c, q, degEps)) return false;
	const Real3 l = barycentric3(a, b, c, q);
	return l[0] >= -eps && l[1] >= -eps && l[2] >= -eps;
}
bool tetrahedronContains(const Real3& a, const Real3& b, const Real3& c, const Real3& d,
                         const Real3& q, real eps) {  // :370-376
	const auto l = barycentric(a, b, c, d, q);
	return l[0] >= -eps && l[1] >= -eps && l[2] >= -eps && l[3] >= -eps;
}
bool solidAngleContains(const Real3& a, const Real3& b, const Real3& c, const Real3& d,
                        const Real3& q, real eps) {  // :410-416
	const auto l = barycentric(a, b, c, d, q);
	return l[0] <= 1 + eps && l[1] >= -eps && l[2] >= -eps && l[3] >= -eps;
}
Real3 oppositeFaceNormal(const Real3& opposite, const Real3& a, const Real3& b, const Real3& c) {
	const Real3 ans = normalize(cross(sub(a, b), sub(c, b)));  // :423-428
	return (dot(ans, sub(a, opposite)) > 0) ? ans : mul(ans, -1);
}
/// geometry.hpp:201-217
Real3 lineWithFlatIntersection(const Real3& f1, const Real3& f2, const Real3& f3, const Real3& l1,
                               const Real3& l2) {
	const Real3 tau = sub(l2, l1), p = sub(f2, f1), q = sub(f3, f1);
	const real A[3][3] = {{tau[0], -p[0], -q[0]}, {tau[1], -p[1], -q[1]}, {tau[2], -p[2], -q[2]}};
	const Real3 params = solve3(A, sub(f1, l1));
	return add(l1, mul(tau, params[0]));
}

uint64_t splitmix(uint64_t x) {
	x += 0x9E3779B97F4A7C15ull;
	x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
	x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
	return x ^ (x >> 31);
}
real unitRandom(uint64_t seed, uint64_t n) {  // [-1, 1)
	return (real)(splitmix(seed * 0x100000001B3ull + n) >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

}  // namespace

// ------------------------------------------------------------------- mesh --

void TetMesh::buildTopology() {
	const int nc = (int)cells.size(), nv = (int)v.size();
	nb.assign(nc, {-1, -1, -1, -1});
	std::map<std::array<int, 3>, std::pair<int, int>> faces;
	for (int c = 0; c < nc; c++)
		for (int i = 0; i < 4; i++) {
			std::array<int, 3> f = {cells[c][(i + 1) % 4], cells[c][(i + 2) % 4], cells[c][(i + 3) % 4]};
			std::sort(f.begin(), f.end());
			auto it = faces.find(f);
			if (it == faces.end()) {
				faces[f] = {c, i};
			} else {
				if (it->second.first < 0) throw Exception("face shared by more than two cells");
				nb[c][i] = it->second.first;
				nb[it->second.first][it->second.second] = c;
				it->second.first = -2;
			}
		}
	std::vector<int> cnt(nv + 1, 0);
	for (const auto& c : cells)
		for (int x : c) cnt[x + 1]++;
	for (int i = 0; i < nv; i++) cnt[i + 1] += cnt[i];
	incOff = cnt;
	incCells.assign(cnt[nv], 0);
	std::vector<int> fill(cnt.begin(), cnt.end() - 1);
	for (int c = 0; c < nc; c++)
		for (int x : cells[c]) incCells[fill[x]++] = c;
}

TetMesh boxMesh(const std::array<int, 3>& n, const Real3& lo, const Real3& hi, real jitter,
                uint64_t seed) {
	for (int i = 0; i < 3; i++)
		if (n[i] < 1 || !(hi[i] > lo[i])) throw Exception("boxMesh: bad box");
	if (!(jitter >= 0 && jitter < 0.25)) throw Exception("boxMesh: jitter must be in [0, 0.25)");
	TetMesh m;
	const int nx = n[0] + 1, ny = n[1] + 1, nz = n[2] + 1;
	auto id = [&](int i, int j, int k) { return (i * ny + j) * nz + k; };
	m.v.resize((size_t)nx * ny * nz);
	for (int i = 0; i < nx; i++)
		for (int j = 0; j < ny; j++)
			for (int k = 0; k < nz; k++) {
				const int ijk[3] = {i, j, k}, nn[3] = {nx, ny, nz};
				Real3 p;
				for (int a = 0; a < 3; a++) {
					const real h = (hi[a] - lo[a]) / n[a];
					p[a] = (ijk[a] == n[a]) ? hi[a] : lo[a] + h * ijk[a];
					const bool onBoundary = ijk[a] == 0 || ijk[a] == nn[a] - 1;
					if (!onBoundary && jitter > 0)
						p[a] += jitter * h * unitRandom(seed, (uint64_t)id(i, j, k) * 3 + a);
				}
				m.v[id(i, j, k)] = p;
			}
	static const int perms[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
	for (int i = 0; i < n[0]; i++)
		for (int j = 0; j < n[1]; j++)
			for (int k = 0; k < n[2]; k++)
				for (const auto& pm : perms) {
					int c[3] = {i, j, k};
					std::array<int, 4> t;
					t[0] = id(c[0], c[1], c[2]);
					for (int s = 0; s < 3; s++) {
						c[pm[s]]++;
						t[s + 1] = id(c[0], c[1], c[2]);
					}
					const real vol = orientedVolume(m.v[t[0]], m.v[t[1]], m.v[t[2]], m.v[t[3]]);
					if (vol < 0) std::swap(t[2], t[3]);
					if (!(vol != 0)) throw Exception("boxMesh: degenerate cell");
					m.cells.push_back(t);
				}
	for (const auto& t : m.cells)
		if (!(orientedVolume(m.v[t[0]], m.v[t[1]], m.v[t[2]], m.v[t[3]]) > 0))
			throw Exception("boxMesh: jitter inverted a cell");
	m.buildTopology();
	return m;
}

// --------------------------------------------------------- triangulation --

bool offContains(const std::vector<Real3>& points, const std::vector<std::array<int, 3>>& faces,
                 const Real3& p) {
	// generalized winding number: sum of the triangles' solid angles / 4 pi
	// (Van Oosterom & Strackee); a point inside k nested closed surfaces gets |k|
	real w = 0;
	for (const auto& f : faces) {
		const Real3 a = sub(points[(size_t)f[0]], p), b = sub(points[(size_t)f[1]], p),
		            c = sub(points[(size_t)f[2]], p);
		const real la = length(a), lb = length(b), lc = length(c);
		const real num = dot(a, cross(b, c));
		const real den = la * lb * lc + dot(a, b) * lc + dot(a, c) * lb + dot(b, c) * la;
		w += 2 * std::atan2(num, den);
	}
	const long k = std::lround(std::fabs(w) / (4 * M_PI));
	return (k % 2) == 1;
}

void readOff(const std::string& fileName, std::vector<Real3>& points,
             std::vector<std::array<int, 3>>& faces) {
	std::ifstream in(fileName);
	if (!in) throw Exception("cannot open " + fileName);
	std::vector<std::string> tokens;
	std::string line;
	while (std::getline(in, line)) {  // '#' starts a comment (meshes/layers_with_fracture.off)
		const size_t h = line.find('#');
		if (h != std::string::npos) line.resize(h);
		std::istringstream ls(line);
		std::string t;
		while (ls >> t) tokens.push_back(t);
	}
	size_t i = 0;
	auto next = [&]() -> const std::string& {
		if (i >= tokens.size()) throw Exception("truncated .off file " + fileName);
		return tokens[i++];
	};
	if (next() != "OFF") throw Exception(fileName + " is not an OFF file");
	const long nv = std::stol(next()), nf = std::stol(next());
	next();  // number of edges
	if (nv < 4 || nf < 4) throw Exception("degenerate .off surface");
	points.assign((size_t)nv, Real3{});
	for (long v = 0; v < nv; v++)
		for (int c = 0; c < 3; c++) points[(size_t)v][c] = std::stod(next());
	faces.clear();
	for (long f = 0; f < nf; f++) {
		if (std::stol(next()) != 3) throw Exception("only triangles are supported in .off");
		std::array<int, 3> t;
		for (int c = 0; c < 3; c++) {
			t[c] = std::stoi(next());
			if (t[c] < 0 || t[c] >= nv) throw Exception("bad .off vertex index");
		}
		faces.push_back(t);
	}
}

void readInm(const std::string& fileName, std::vector<Real3>& points,
             std::vector<std::array<int, 4>>& cells, std::vector<int>& materials) {
	std::ifstream in(fileName);
	if (!in) throw Exception("cannot open " + fileName);
	auto fields = [](const std::string& line) {
		std::istringstream ls(line);
		std::vector<std::string> out;
		std::string t;
		while (ls >> t) out.push_back(t);
		return out;
	};
	std::string line;
	auto next = [&]() {
		if (!std::getline(in, line)) throw Exception("truncated INM mesh file " + fileName);
		return fields(line);
	};
	auto f = next();  // readPoints (:121-141)
	if (f.size() != 1) throw Exception("INM: number of points expected");
	const long np = std::stol(f[0]);
	if (np < 4) throw Exception("INM: fewer points than a cell has");
	points.assign((size_t)np, Real3{});
	for (long i = 0; i < np; i++) {
		f = next();
		if (f.size() != 3) throw Exception("INM: a point needs 3 coordinates");
		for (int c = 0; c < 3; c++) points[(size_t)i][c] = std::stod(f[(size_t)c]);
	}
	f = next();  // readCells (:144-164)
	if (f.size() != 1) throw Exception("INM: number of cells expected");
	const long nc = std::stol(f[0]);
	if (nc < 1) throw Exception("INM: no cells");
	cells.clear();
	materials.clear();
	for (long i = 0; i < nc; i++) {
		f = next();
		if (f.size() != 5) throw Exception("INM: a cell needs 4 vertices and a material");
		std::array<int, 4> c;
		for (int k = 0; k < 4; k++) {
			c[k] = std::stoi(f[(size_t)k]);
			if (c[k] < 1 || c[k] > np) throw Exception("INM: cell vertex out of range");
		}
		cells.push_back(c);
		materials.push_back(std::stoi(f[4]));
	}
	f = next();  // checkEndOfFile (:167-172)
	if (f.size() != 1 || std::stoi(f[0]) != 0) throw Exception("INM: the file must end with 0");
}

namespace {
/// The INM mesher: the file's cells are the triangulation (the reference inserts
/// the points into a CGAL Delaunay triangulation and gives each of its cells the
/// material of the same INM cell, InmMeshLoader.hpp:47-93; CGAL is absent, so the
/// file must hold the whole tetrahedralisation), grid id = material.
Triangulation inmTriangulation(const Task& task) {
	std::vector<Real3> pts;
	std::vector<std::array<int, 4>> cells;
	std::vector<int> mats;
	readInm(task.simplexGrid.fileName, pts, cells, mats);
	Triangulation tr;
	tr.all.v = pts;
	for (auto c : cells) {
		for (int& x : c) x -= 1;  // INM numbers vertices from 1
		const real vol = orientedVolume(pts[(size_t)c[0]], pts[(size_t)c[1]], pts[(size_t)c[2]],
		                                pts[(size_t)c[3]]);
		if (!(vol != 0)) throw Exception("INM: degenerate cell");
		if (vol < 0) std::swap(c[2], c[3]);
		tr.all.cells.push_back(c);
	}
	tr.all.buildTopology();
	for (int m : mats) {
		if (!task.bodies.count((size_t)m)) throw Exception("INM: a cell's material names no body");
		tr.gridId.push_back(m);
	}
	return tr;
}
}  // namespace

Triangulation buildTriangulation(const Task& task) {
	const auto& sg = task.simplexGrid;
	if (task.bodies.empty()) throw Exception("the simplex task has no bodies");
	if (sg.mesher == Task::SimplexGrid::Mesher::INM_MESHER) {
		if (!sg.offFaces.empty() || !sg.bodyAreas.empty())
			throw Exception("INM meshes carry their own cells and grid ids");
		return inmTriangulation(task);
	}
	Triangulation tr;
	tr.all = boxMesh(sg.cells, sg.lo, sg.hi, sg.jitter, sg.seed);
	const int firstBody = (int)task.bodies.begin()->first;
	tr.gridId.assign(tr.all.cells.size(), firstBody);
	for (size_t c = 0; c < tr.all.cells.size(); c++) {
		const auto& t = tr.all.cells[c];
		Real3 ctr = add(add(add(tr.all.v[(size_t)t[0]], tr.all.v[(size_t)t[1]]), tr.all.v[(size_t)t[2]]),
		                tr.all.v[(size_t)t[3]]);
		ctr = mul(ctr, 0.25);
		if (!sg.offFaces.empty() && !offContains(sg.offPoints, sg.offFaces, ctr)) {
			tr.gridId[c] = EMPTY_SPACE;
			continue;
		}
		for (const auto& rule : sg.bodyAreas) {
			if (!task.bodies.count(rule.second)) throw Exception("body area names an unknown body");
			if (rule.first->contains(ctr)) tr.gridId[c] = (int)rule.second;
		}
	}
	return tr;
}

TetMesh bodyMesh(const Triangulation& tr, int id) {
	const TetMesh& all = tr.all;
	const int nvAll = all.nVertices();
	// vertices on the box surface touch the (infinite) empty space
	std::vector<char> onHull((size_t)nvAll, 0);
	for (size_t c = 0; c < all.cells.size(); c++)
		for (int i = 0; i < 4; i++)
			if (all.nb[c][i] < 0)
				for (int k = 1; k < 4; k++) onHull[(size_t)all.cells[c][(i + k) % 4]] = 1;
	std::vector<int> cellsOf;
	std::vector<int> local((size_t)nvAll, -1);
	for (size_t c = 0; c < all.cells.size(); c++)
		if (tr.gridId[c] == id) {
			cellsOf.push_back((int)c);
			for (int x : all.cells[c]) local[(size_t)x] = 0;
		}
	if (cellsOf.empty()) throw Exception("a body without cells");
	TetMesh m;
	for (int g = 0; g < nvAll; g++)
		if (local[(size_t)g] == 0) {
			local[(size_t)g] = (int)m.v.size();
			m.v.push_back(all.v[(size_t)g]);
			m.global.push_back(g);
		}
	for (int c : cellsOf) {
		std::array<int, 4> t;
		for (int i = 0; i < 4; i++) t[i] = local[(size_t)all.cells[(size_t)c][i]];
		m.cells.push_back(t);
	}
	m.buildTopology();
	m.nbGrid.assign(m.cells.size(), {id, id, id, id});
	for (size_t lc = 0; lc < cellsOf.size(); lc++)
		for (int i = 0; i < 4; i++)
			if (m.nb[lc][i] < 0) {
				const int gn = all.nb[(size_t)cellsOf[lc]][i];
				m.nbGrid[lc][i] = gn < 0 ? EMPTY_SPACE : tr.gridId[(size_t)gn];
				if (m.nbGrid[lc][i] == id) throw Exception("bodyMesh: lost a face neighbour");
			}
	m.otherGrids.assign(m.v.size(), {});
	for (int lv = 0; lv < m.nVertices(); lv++) {
		const int g = m.global[(size_t)lv];
		std::set<int> s;
		if (onHull[(size_t)g]) s.insert(EMPTY_SPACE);
		for (int p = all.incOff[(size_t)g]; p < all.incOff[(size_t)g + 1]; p++) {
			const int gid = tr.gridId[(size_t)all.incCells[(size_t)p]];
			if (gid != id) s.insert(gid);
		}
		m.otherGrids[(size_t)lv].assign(s.begin(), s.end());
	}
	return m;
}

// ------------------------------------------------------------------- grid --

Grid::Grid(const TetMesh& m) : mesh(m) {
	const int nv = m.nVertices();
	if (m.otherGrids.size() != (size_t)nv || m.nbGrid.size() != m.cells.size())
		throw Exception("Grid: the mesh was not cut out of a triangulation (bodyMesh)");
	inner.assign(nv, 1);
	// borderState (SimplexGrid.hpp:388-395) + markInnersAndBorders (SimplexGrid.cpp:216-252)
	for (int it = 0; it < nv; it++) {
		const auto& o = m.otherGrids[(size_t)it];
		if (o.empty()) {
			innerIdx.push_back(it);
			continue;
		}
		inner[it] = 0;
		if (o.size() == 1 && o[0] != EMPTY_SPACE) contactIdx.push_back(it);
		else borderIdx.push_back(it);  // BORDER or MULTICONTACT
	}
	// collectCellHeightsStatistics (SimplexGrid.cpp:266-285): Histogram of 100 bins
	std::vector<real> hs;
	for (const auto& t : m.cells) hs.push_back(minimalHeight4(P(t[0]), P(t[1]), P(t[2]), P(t[3])));
	const real mn = *std::min_element(hs.begin(), hs.end());
	const real mx = *std::max_element(hs.begin(), hs.end());
	const size_t nBins = 100;
	std::vector<size_t> bins;
	const real binSize0 = (mx - mn) / real(nBins);
	if (mx == mn) {  // Histogram.hpp:13-33
		bins.assign(nBins, 0);
		bins[0] = hs.size();
	} else {
		bins.assign(nBins + 1, 0);
		for (real h : hs) ++bins[(size_t)((h - mn) / binSize0)];
		bins[nBins - 1] += bins.back();
		bins.pop_back();
	}
	const real binSize = (mx - mn) / (real)bins.size();  // Histogram.hpp:44-58
	real ip = 0, cnt = 0;
	for (size_t i = 0; i < bins.size(); i++) {
		ip = ip + (real)bins[i] * (mn + (real(i) + 0.5) * binSize);
		cnt = cnt + (real)bins[i];
	}
	averageHeight = ip / cnt;
	minimalHeight = mn;
}

template <typename Pred>
Real3 Grid::normal(int it, Pred use) const {
	Real3 sum = {0, 0, 0};
	bool any = false;
	for (int p = mesh.incOff[it]; p < mesh.incOff[it + 1]; p++) {
		const int c = mesh.incCells[p];
		for (int i = 0; i < 4; i++) {
			if (mesh.nb[c][i] >= 0 || mesh.cells[c][i] == it) continue;  // face must contain it
			if (!use(mesh.nbGrid[c][i])) continue;
			const auto& t = mesh.cells[c];
			sum = add(sum, oppositeFaceNormal(P(t[i]), P(t[(i + 1) % 4]), P(t[(i + 2) % 4]),
			                                  P(t[(i + 3) % 4])));  // Cgal3DTriangulation.hpp:109-118
			any = true;
		}
	}
	if (!any) return {0, 0, 0};
	return normalize(sum);
}
Real3 Grid::borderNormal(int it) const {
	return normal(it, [](int g) { return g == EMPTY_SPACE; });
}
Real3 Grid::contactNormal(int it, int other) const {
	return normal(it, [other](int g) { return g == other; });
}
Real3 Grid::commonNormal(int it) const {
	return normal(it, [](int) { return true; });
}

std::vector<int> Grid::neighborVertices(int it) const {
	std::set<int> s;
	for (int p = mesh.incOff[it]; p < mesh.incOff[it + 1]; p++)
		for (int x : mesh.cells[mesh.incCells[p]]) s.insert(x);
	s.erase(it);
	return std::vector<int>(s.begin(), s.end());
}

int Grid::otherVertexIndex(int cell, int a, int b, int c) const {  // Cgal3DTriangulation.hpp:272-280
	for (int i = 0; i < 4; i++) {
		const int d = mesh.cells[cell][i];
		if (d != a && d != b && d != c) return i;
	}
	throw Exception("Cell contains equal vertices");
}

int Grid::findCrossedIncidentCell(int vh, const Real3& query, real eps) const {  // :221-238
	for (int p = mesh.incOff[vh]; p < mesh.incOff[vh + 1]; p++) {
		const int cand = mesh.incCells[p];
		const auto& t = mesh.cells[cand];
		const int a = t[otherVertexIndex(cand, vh, vh, vh)];
		const int b = t[otherVertexIndex(cand, vh, vh, a)];
		const int c = t[otherVertexIndex(cand, vh, a, b)];
		if (solidAngleContains(P(vh), P(a), P(b), P(c), query, eps)) return cand;
	}
	return -1;
}

void Grid::findCrossedInsideOutFacet(int t, const Real3& q, const Real3& p, int& a, int& b, int& c,
                                     real eps) const {  // :247-259
	a = b = c = -1;
	for (int i = 0; i < 4; i++) {
		const int a1 = mesh.cells[t][(i + 1) % 4], b1 = mesh.cells[t][(i + 2) % 4],
		          c1 = mesh.cells[t][(i + 3) % 4];
		if (solidAngleContains(q, P(a1), P(b1), P(c1), p, eps)) {
			a = a1;
			b = b1;
			c = c1;
			return;
		}
	}
}

// LineWalker<Triangulation, 3>::collectCells (LineWalker.hpp:25-52).  Leaving
// the body is the step onto nb == -1; the face crossed then is {u, v, w}.
std::vector<int> Grid::collectCells(const Real3& q, const Real3& p, int t, int u, int v, int w,
                                    std::array<int, 3>& lastFace) const {
	std::vector<int> ans;
	ans.push_back(t);
	auto orient = [&](const Real3& a, const Real3& b, const Real3& c, const Real3& d) {
		return orientedVolume(a, b, c, d);
	};
	while (orient(P(u), P(v), P(w), p) < 0) {
		const int nt = mesh.nb[t][otherVertexIndex(t, u, v, w)];  // neighborThrough
		if (nt < 0) {
			lastFace = {u, v, w};
			ans.push_back(-1);
			break;
		}
		t = nt;
		ans.push_back(t);
		const int s = mesh.cells[t][otherVertexIndex(t, u, v, w)];
		if (orient(P(u), P(s), q, p) > 0) {
			if (orient(P(v), P(s), q, p) > 0) u = s;
			else w = s;
		} else {
			if (orient(P(w), P(s), q, p) > 0) v = s;
			else u = s;
		}
	}
	return ans;
}

std::vector<int> Grid::cellsAlongSegmentFromVertex(int q, const Real3& p,
                                                   std::array<int, 3>& lastFace) const {
	const int t = findCrossedIncidentCell(q, p, 0);  // LineWalker.hpp:54-69
	if (t < 0) return {};
	const auto& c = mesh.cells[t];
	int u = c[otherVertexIndex(t, q, q, q)];
	int v = c[otherVertexIndex(t, q, q, u)];
	const int w = c[otherVertexIndex(t, q, u, v)];
	if (orientedVolume(P(u), P(v), P(w), P(q)) < 0) std::swap(u, v);
	return collectCells(P(q), p, t, u, v, w, lastFace);
}

std::vector<int> Grid::cellsAlongSegmentFromCell(int t, const Real3& q, const Real3& p,
                                                 std::array<int, 3>& lastFace) const {
	int u, v, w;  // LineWalker.hpp:71-88
	findCrossedInsideOutFacet(t, q, p, u, v, w, 0);
	if (u < 0) findCrossedInsideOutFacet(t, q, p, u, v, w, EQUALITY_TOLERANCE);
	if (u < 0) return {};
	if (orientedVolume(P(u), P(v), P(w), q) < 0) std::swap(u, v);
	return collectCells(q, p, t, u, v, w, lastFace);
}

// SimplexGrid.cpp:115-164
Grid::Cell Grid::checkLineWalkFoundCell(int it, const std::vector<int>& cells,
                                        const std::array<int, 3>& lastFace, const Real3& start,
                                        const Real3& query) const {
	Cell none;
	if (cells.empty()) return none;
	auto contains = [&](int c) {
		const auto& t = mesh.cells[c];
		return tetrahedronContains(P(t[0]), P(t[1]), P(t[2]), P(t[3]), query, EQUALITY_TOLERANCE);
	};
	auto full = [&](int c) {
		Cell r;
		r.n = 4;
		for (int i = 0; i < 4; i++) r.v[i] = mesh.cells[c][i];
		return r;
	};
	const int last = cells.back();
	if (last >= 0 && contains(last)) return full(last);
	if (cells.size() == 1) {
		if (isInner(it)) throw Exception("line walk: inner node with a one-cell walk");
		return none;
	}
	const int prev = cells[cells.size() - 2];
	if (contains(prev)) return full(prev);
	if (!isInner(it)) return none;
	if (last < 0) {
		// Triangulation::commonVertices(prev, last): prev's vertices in cell order
		std::vector<int> face;
		for (int i = 0; i < 4; i++) {
			const int x = mesh.cells[prev][i];
			if (x == lastFace[0] || x == lastFace[1] || x == lastFace[2]) face.push_back(x);
		}
		// filterFaceNotCrossedByTheRay (Cgal3DTriangulation.hpp:183-213)
		std::vector<int> f;
		const Real3 p0 = P(face[0]), p1 = P(face[1]), p2 = P(face[2]);
		const Real3 x = lineWithFlatIntersection(p0, p1, p2, start, query);
		const Real3 ps[3] = {p0, p1, p2};
		if (triangleContains(p0, p1, p2, x, EQUALITY_TOLERANCE, EQUALITY_TOLERANCE)) {
			f = face;
		} else {
			for (int i = 0; i < 3 && f.empty(); i++)
				for (int j = i + 1; j < 3 && f.empty(); j++)
					if (segmentContains(ps[i], ps[j], x, EQUALITY_TOLERANCE, EQUALITY_TOLERANCE))
						f = {face[i], face[j]};
			for (int i = 0; i < 3 && f.empty(); i++)
				if (segmentContains(start, query, ps[i], EQUALITY_TOLERANCE, EQUALITY_TOLERANCE))
					f = {face[i]};
		}
		Cell r;
		r.n = (int)f.size();
		for (int i = 0; i < r.n; i++) r.v[i] = f[i];
		return r;
	}
	return none;
}

// SimplexGrid.cpp:57-112
Grid::Cell Grid::findCellCrossedByTheRay(int it, const Real3& shift) const {
	const Real3 start = P(it);
	const Real3 query = add(start, shift);
	std::array<int, 3> lastFace = {-1, -1, -1};
	std::vector<int> along = cellsAlongSegmentFromVertex(it, query, lastFace);
	Cell found = checkLineWalkFoundCell(it, along, lastFace, start, query);
	if (found.n > 0) return found;
	int startCell = findCrossedIncidentCell(it, query, 0);
	if (startCell < 0) startCell = findCrossedIncidentCell(it, query, EQUALITY_TOLERANCE);
	if (startCell < 0) startCell = mesh.incCells[mesh.incOff[it]];
	const auto& t = mesh.cells[startCell];
	// Triangulation::center (Cgal3DTriangulation.hpp:263-269): (a + b + c + d) / 4
	Real3 center = add(add(add(P(t[0]), P(t[1])), P(t[2])), P(t[3]));
	center = {center[0] / 4, center[1] / 4, center[2] / 4};
	constexpr real w = 1e-3;
	const Real3 startPoint = add(mul(center, w), mul(start, 1 - w));
	lastFace = {-1, -1, -1};
	along = cellsAlongSegmentFromCell(startCell, startPoint, query, lastFace);
	found = checkLineWalkFoundCell(it, along, lastFace, start, query);
	if (found.n > 0) return found;
	if (isInner(it)) throw Exception("line walk failed for an inner node");
	return Cell();
}

// ------------------------------------------------------------------- plans --

GradientPlan buildGradientPlan(const Grid& grid) {
	const auto& m = grid.mesh;
	const int nv = m.nVertices();
	GradientPlan g;
	g.offsets.push_back(0);
	for (int it = 0; it < nv; it++) {
		const std::vector<int> nbs = grid.neighborVertices(it);
		const int K = std::min((int)nbs.size(), MAX_NUMBER_OF_NEIGHBOR_VERTICES);
		real A[MAX_NUMBER_OF_NEIGHBOR_VERTICES][3] = {};
		real W[MAX_NUMBER_OF_NEIGHBOR_VERTICES] = {};
		for (int i = 0; i < K; i++) {
			const Real3 d = sub(m.v[nbs[i]], m.v[it]);
			for (int c = 0; c < 3; c++) A[i][c] = d[c];
			W[i] = 1.0 / length(d);
			g.neighbors.push_back(nbs[i]);
			for (int c = 0; c < 3; c++) g.rows.push_back(d[c]);
			g.weights.push_back(W[i]);
		}
		g.offsets.push_back((int)g.neighbors.size());
		// transposeMultiply(A, W * A) over all MAX rows (functions.hpp:220-234)
		real M[3][3];
		for (int r = 0; r < 3; r++)
			for (int c = 0; c < 3; c++) {
				real s = A[0][r] * (W[0] * A[0][c]);
				for (int n = 1; n < MAX_NUMBER_OF_NEIGHBOR_VERTICES; n++) s += A[n][r] * (W[n] * A[n][c]);
				M[r][c] = s;
				g.M.push_back(s);
			}
		const real det = det3(M[0][0], M[0][1], M[0][2], M[1][0], M[1][1], M[1][2], M[2][0], M[2][1],
		                      M[2][2]);
		if (det == 0) throw Exception("estimateGradient: SLE determinant is zero");
		g.det.push_back(det);
	}
	return g;
}

std::array<real, 4> barycentricCoordinates(const Real3& a, const Real3& b, const Real3& c, const Real3& d,
                                           const Real3& q) {
	return barycentric(a, b, c, d, q);
}

void interpolateInOwnerPick(const Real3 (&pts)[6], const Real3& q, int (&slot)[4], real (&lam)[4]) {
	// TetrahedronInterpolator::interpolateInOwner (hpp:113-155): the 15 tetrahedra
	// in the reference's TRY_TETRAHEDRON order, the first non-degenerate one whose
	// barycentrics pass isInterpolation (hpp:15-20)
	static const int tries[15][4] = {{0, 1, 2, 3}, {0, 1, 2, 4}, {0, 1, 2, 5}, {0, 1, 3, 4}, {0, 1, 3, 5},
	                                 {0, 1, 4, 5}, {0, 2, 3, 4}, {0, 2, 3, 5}, {0, 2, 4, 5}, {0, 3, 4, 5},
	                                 {1, 2, 3, 4}, {1, 2, 3, 5}, {1, 2, 4, 5}, {1, 3, 4, 5}, {2, 3, 4, 5}};
	for (const auto& tr : tries) {
		if (volume(pts[tr[0]], pts[tr[1]], pts[tr[2]], pts[tr[3]]) == 0) continue;
		const auto l = barycentric(pts[tr[0]], pts[tr[1]], pts[tr[2]], pts[tr[3]], q);
		if (l[0] > -EQUALITY_TOLERANCE && l[1] > -EQUALITY_TOLERANCE && l[2] > -EQUALITY_TOLERANCE &&
		    l[3] > -EQUALITY_TOLERANCE) {
			for (int i = 0; i < 4; i++) {
				slot[i] = tr[i];
				lam[i] = l[i];
			}
			return;
		}
	}
	throw Exception("Containing tetrahedron is not found");  // THROW_INVALID_ARG, hpp:153
}

StagePlan buildStagePlan(const Grid& grid, const Real3& direction, const real L[9], real tau) {
	const auto& m = grid.mesh;
	const int nv = m.nVertices();
	StagePlan plan;
	plan.feet.assign((size_t)nv * 6, gsx_foot{});
	plan.outerCode.assign((size_t)nv, 0);
	// contactAndBorderStage: contact nodes, then border nodes (hpp:90-95)
	plan.borderNodes = grid.contactIdx;
	plan.borderNodes.insert(plan.borderNodes.end(), grid.borderIdx.begin(), grid.borderIdx.end());
	plan.innerNodes = grid.innerIdx;
	static const std::vector<int> RIGHT = {1, 3, 5}, LEFT = {0, 2, 4};  // Model.cpp:81-82
	for (int it = 0; it < nv; it++) {
		const bool innerNode = grid.isInner(it);
		std::vector<int> outer;
		for (int k = 0; k < 6; k++) {
			gsx_foot& f = plan.feet[(size_t)it * 6 + k];
			const real dx = -tau * L[k];  // crossingPoints (common.hpp:46-52)
			if (dx == 0) throw Exception("zero crossing point for a wave invariant");
			const Real3 shift = mul(direction, dx);
			for (int r = 0; r < 3; r++) plan.shift[k][r] = shift[r];
			const Grid::Cell t = grid.findCellCrossedByTheRay(it, shift);
			const Real3 q = add(m.v[it], shift);
			if (t.n == 4) {
				f.kind = GSX_FOOT_CELL;
				const auto lam = barycentric(m.v[t.v[0]], m.v[t.v[1]], m.v[t.v[2]], m.v[t.v[3]], q);
				for (int i = 0; i < 4; i++) {
					// TetrahedronInterpolator::isInterpolation assert (hpp:15-20)
					if (!(lam[i] > -EQUALITY_TOLERANCE)) throw Exception("foot outside its cell");
					f.v[i] = t.v[i];
					f.lam[i] = lam[i];
				}
				for (int c = 0; c < 3; c++) f.q[c] = q[c];
			} else if (t.n == 0 || ((t.n == 3 || t.n == 2) && !innerNode)) {
				f.kind = GSX_FOOT_OUTER;
				outer.push_back(k);
			} else if (t.n == 3) {
				// interpolateInSpaceTime (common.hpp:102-129): the geometry is static
				const Real3 r0 = m.v[it], r1 = m.v[t.v[0]], r2 = m.v[t.v[1]], r3 = m.v[t.v[2]];
				const Real3 rc = lineWithFlatIntersection(r1, r2, r3, r0, add(r0, shift));
				const auto w = lls32(sub(r2, r1), sub(r3, r1), sub(rc, r1));
				const Real3 pts[6] = {{0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {0, 1, 1}};
				const Real3 qst = {w[0], w[1], 1 - length(sub(rc, r0)) / length(shift)};
				real lam[4];
				interpolateInOwnerPick(pts, qst, f.slot, lam);  // throws when none contains qst
				for (int i = 0; i < 4; i++) f.lam[i] = lam[i];
				f.kind = GSX_FOOT_SPACETIME;
				for (int i = 0; i < 3; i++) f.v[i] = t.v[i];
			} else if (t.n == 2) {
				// interpolateInSpaceTime1D in 3-D (GridCharacteristicMethodInRiemannInvariants.hpp:296-303)
				throw Exception("This did not occur ever before");
			} else {
				f.kind = GSX_FOOT_ZERO;  // n == 1: no branch assigns u (hpp:168-196)
			}
		}
		if (innerNode) {
			if (!outer.empty()) throw Exception("outer invariant at an inner node");  // hpp:119
			continue;
		}
		// contactAndBorderStage's outer-invariant completion (hpp:71-86)
		if (outer != RIGHT && outer != LEFT && outer.size() != 6 && !outer.empty()) {
			auto inter = [](const std::vector<int>& a, const std::vector<int>& b) {
				std::vector<int> r;
				std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(r));
				return r;
			};
			auto uni = [](const std::vector<int>& a, const std::vector<int>& b) {
				std::vector<int> r;
				std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(r));
				return r;
			};
			if (!inter(outer, RIGHT).empty()) outer = uni(outer, RIGHT);
			if (!inter(outer, LEFT).empty()) outer = uni(outer, LEFT);
			for (int k : outer) plan.feet[(size_t)it * 6 + k].kind = GSX_FOOT_OUTER;
		}
		if (outer == RIGHT) plan.outerCode[it] = 1;
		else if (outer == LEFT) plan.outerCode[it] = 2;
		else if (!outer.empty()) plan.outerCode[it] = 3;  // all six after the completion
	}
	return plan;
}

std::array<real, 27> borderMatrix(BorderConditions::T type, const Real3& normal) {
	std::array<real, 27> B{};
	real S[3][3];
	detail::localBasisOf<3>(normal.data(), S);
	if (type == BorderConditions::T::FIXED_FORCE) {
		// G_k(i, j) += S(i, k) p(j) over a SymmetricMatrix (Symmetry.hpp:38-46), so
		// an off-diagonal slot collects both (i, j) and (j, i); setSigma copies it.
		for (int k = 0; k < 3; k++) {
			real G[6] = {0, 0, 0, 0, 0, 0};
			for (int i = 0; i < 3; i++)
				for (int j = 0; j < 3; j++) {
					const int a = std::min(i, j), b = std::max(i, j);
					G[a * 3 - ((a - 1) * a) / 2 + b - a] += S[i][k] * normal[j];
				}
			for (int q = 0; q < 6; q++) B[(size_t)k * 9 + 3 + q] = G[q];
		}
	} else {
		for (int i = 0; i < 3; i++)
			for (int j = 0; j < 3; j++) B[(size_t)i * 9 + j] = S[j][i];  // setVelocity(S column i)
	}
	return B;
}

namespace {
/// calculateOuterWaveCorrection's |det(B * Omega)| (common.hpp:186-202)
real outerDeterminantFabs(const std::array<real, 27>& B, const std::array<real, 81>& U1,
                          const int cols[3]) {
	real M[3][3];
	for (int i = 0; i < 3; i++)
		for (int j = 0; j < 3; j++) {
			real x = B[(size_t)i * 9 + 0] * U1[(size_t)0 * 9 + cols[j]];
			for (int n = 1; n < 9; n++) x += B[(size_t)i * 9 + n] * U1[(size_t)n * 9 + cols[j]];
			M[i][j] = x;
		}
	return std::fabs(det3(M[0][0], M[0][1], M[0][2], M[1][0], M[1][1], M[1][2], M[2][0], M[2][1],
	                      M[2][2]));
}
}  // namespace

BorderPlan buildBorderPlan(const Task& task, const Grid& grid, const GcmMatrices<3>& matrices,
                           const real calc[3][3], const StagePlan stages[3]) {
	BorderPlan bp;
	const auto& conds = task.borderConditions;
	if (conds.size() > GSX_MAX_BORDER_CONDITIONS) throw Exception("too many border conditions");
	for (const auto& c : conds) {
		if (!c.area) throw Exception("border condition without area");
		if (c.values.size() != 3) throw Exception("border condition needs OUTER_NUMBER = 3 values");
		bp.type.push_back(c.type == BorderConditions::T::FIXED_FORCE ? GSX_FIXED_FORCE
		                                                             : GSX_FIXED_VELOCITY);
	}
	std::vector<int> count(conds.size(), 0);
	for (int it : grid.borderIdx) {  // Engine::addBorderNode (Engine.cpp:292-309)
		const Real3 bn = grid.borderNormal(it);
		const bool isMulticontact = bn[0] == 0 && bn[1] == 0 && bn[2] == 0;
		int chosen = -1;
		for (size_t c = 0; c < conds.size(); c++)
			if (conds[c].area->contains(grid.mesh.v[it]) &&
			    (!isMulticontact || conds[c].useForMulticontactNodes))
				chosen = (int)c;
		if (chosen < 0) continue;
		const Real3 n = grid.commonNormal(it);
		if (n[0] == 0 && n[1] == 0 && n[2] == 0) throw Exception("zero common normal at a border node");
		bp.nodes.push_back(it);
		bp.cond.push_back(chosen);
		count[(size_t)chosen]++;
		for (int r = 0; r < 3; r++) bp.normal.push_back(n[r]);
		const auto B = borderMatrix(conds[(size_t)chosen].type, n);
		bp.B.insert(bp.B.end(), B.begin(), B.end());
		real S[3][3];
		detail::localBasisOf<3>(n.data(), S);
		for (int r = 0; r < 3; r++)
			for (int c = 0; c < 3; c++) bp.S.push_back(S[r][c]);
	}
	const size_t nn = bp.nodes.size();
	bp.outer.assign(3 * nn, 0);
	for (int s = 0; s < 3; s++)
		for (size_t i = 0; i < nn; i++) bp.outer[s * nn + i] = stages[s].outerCode[(size_t)bp.nodes[i]];
	// getMaximalPossibleDeterminant (BorderCorrector.hpp:198-214): B along the stage
	// direction, RIGHT outer columns; the correction's threshold is 1e-3 of it.
	static const int RIGHT[3] = {1, 3, 5};
	bp.minDet.assign(3 * conds.size(), 0.0);
	for (size_t c = 0; c < conds.size(); c++) {
		if (!count[c]) continue;  // applyInGlobalBasis returns before (hpp:124)
		for (int s = 0; s < 3; s++) {
			const Real3 dir = {calc[0][s], calc[1][s], calc[2][s]};
			const real det = outerDeterminantFabs(borderMatrix(conds[c].type, dir), matrices.m[s].U1, RIGHT);
			if (!(det > 0)) throw Exception("degenerate outer-wave system along the stage direction");
			bp.minDet[c * 3 + s] = 1e-3 * det;
		}
	}
	return bp;
}

}  // namespace simplex
}  // namespace gcm

// ------------------------------------------------------------------ engine --
namespace gcm {
namespace simplex {

namespace {
void calcBasis(const Task& task, real calc[3][3]) {
	if (task.calculationBasis.size() != 9)  // Engine.hpp:186-197 (random basis: not on this path)
		throw Exception("the simplex path needs a constant 3x3 calculation basis");
	for (int r = 0; r < 3; r++)
		for (int c = 0; c < 3; c++) calc[r][c] = task.calculationBasis[(size_t)r * 3 + c];
}
}  // namespace

namespace {

/// The set-up of one body (Engine::createMeshes, Engine.cpp:53-93 + the mesh's
/// setUpPde): grid, matrices of its material, plans, initial state.
BodyPlans buildBody(const Task& task, const Triangulation& tr, size_t id, const real calc[3][3]) {
	const auto& body = task.bodies.at(id);
	if (body.materialId != Materials::T::ISOTROPIC || body.modelId != Models::T::ELASTIC)
		throw Exception("only isotropic elastic bodies are on this path");
	if (!body.odes.empty()) throw Exception("ODEs are not on the simplex path");
	if (!task.materialConditions.byBodies.bodyMaterialMap.count(id))
		throw Exception("no material for a simplex body");
	const auto mat = task.materialConditions.byBodies.bodyMaterialMap.at(id);
	BodyPlans p;
	p.id = id;
	p.mesh = bodyMesh(tr, (int)id);
	Grid grid(p.mesh);
	ElasticModel<3>::constructGcmMatrices(p.matrices, *mat, calc);
	p.maximalEigenvalue = p.matrices.getMaximalEigenvalue();
	p.averageHeight = grid.averageHeight;
	p.gradient = buildGradientPlan(grid);
	p.borderIdx = grid.borderIdx;
	p.innerIdx = grid.innerIdx;
	p.contactIdx = grid.contactIdx;
	// InitialCondition::apply (util/task/InitialCondition.hpp:23-88): vectors and quantities
	if (!task.initialCondition.waves.empty())
		throw Exception("wave initial conditions are not on the simplex path");
	std::vector<std::pair<std::shared_ptr<Area>, std::array<real, 9>>> ics;
	for (const auto& v : task.initialCondition.vectors) {
		if (v.list.size() != 9) throw Exception("initial vector has the wrong size");
		std::array<real, 9> a;
		std::copy(v.list.begin(), v.list.end(), a.begin());
		ics.push_back({v.area, a});
	}
	for (const auto& q : task.initialCondition.quantities) {
		std::array<real, 9> a{};
		setQuantity(3, q.physicalQuantity, q.value, a.data());
		ics.push_back({q.area, a});
	}
	const int nv = p.mesh.nVertices();
	p.pde.assign((size_t)nv * 9, 0.0);
	for (int it = 0; it < nv; it++) {
		real* v = &p.pde[(size_t)it * 9];
		for (const auto& ic : ics)
			if (ic.first->contains(p.mesh.v[it]))
				for (int c = 0; c < 9; c++) v[c] += ic.second[c];
	}
	return p;
}

int outerSize(int code) { return code == 0 ? 0 : code == 3 ? 6 : 3; }

/// ContactCorrectorInRiemannInvariants::matchInnersAndOuters (ContactCorrector.hpp:365-397)
/// on the stage's wave-index codes (0 none, 1 RIGHT, 2 LEFT, 3 both).
void matchInnersAndOuters(int& a, int& b, bool& zeroed) {
	const int N = (outerSize(a) + outerSize(b)) / 3;
	zeroed = false;
	if (N % 2 == 0) return;
	if (N == 3) {
		a = b = 3;
	} else {
		if (a == 0) a = (b == 2) ? 1 : 2;  // B LEFT -> A RIGHT, B RIGHT -> A LEFT
		else b = (a == 2) ? 1 : 2;
	}
	zeroed = true;
}

/// Engine::createContacts (Engine.cpp:220-248) + addBorderOrContact / addContactNode
/// (:252-287) for one pair of bodies, and the per-stage data of the corrector.
ContactPlan buildContact(const Task& task, const Triangulation& tr, const std::vector<BodyPlans>& bodies,
                         size_t ia, size_t ib, const real calc[3][3]) {
	ContactPlan cp;
	cp.a = ia;
	cp.b = ib;
	const BodyPlans& A = bodies[ia];
	const BodyPlans& B = bodies[ib];
	cp.condition = task.contactCondition.defaultCondition;
	const auto key = std::make_pair(A.id, B.id);
	if (task.contactCondition.gridToGridConditions.count(key))
		cp.condition = task.contactCondition.gridToGridConditions.at(key);
	// ContactCorrectorFactory (ContactCorrector.hpp:506-552): ADHESION needs elastic
	// bodies, SLIDE acoustic ones (not on this path)
	if (cp.condition != ContactConditions::T::ADHESION)
		throw Exception("only ADHESION contacts between elastic bodies are supported");
	Grid gA(A.mesh), gB(B.mesh);
	std::vector<int> localA((size_t)tr.all.nVertices(), -1), localB((size_t)tr.all.nVertices(), -1);
	for (int i = 0; i < A.mesh.nVertices(); i++) localA[(size_t)A.mesh.global[(size_t)i]] = i;
	for (int i = 0; i < B.mesh.nVertices(); i++) localB[(size_t)B.mesh.global[(size_t)i]] = i;
	for (int g = 0; g < tr.all.nVertices(); g++) {  // triangulation vertex order
		const int la = localA[(size_t)g], lb = localB[(size_t)g];
		if (la < 0 || lb < 0) continue;
		const auto& o = A.mesh.otherGrids[(size_t)la];
		if (o.size() != 1 || o[0] != (int)B.id) continue;  // incidentGrids == {A, B}
		const Real3 n = gA.contactNormal(la, (int)B.id);
		if (n[0] == 0 && n[1] == 0 && n[2] == 0) continue;
		cp.nodesA.push_back(la);
		cp.nodesB.push_back(lb);
		for (int r = 0; r < 3; r++) cp.normal.push_back(n[r]);
		real S[3][3];
		detail::localBasisOf<3>(n.data(), S);
		for (int r = 0; r < 3; r++)
			for (int c = 0; c < 3; c++) cp.S.push_back(S[r][c]);
	}
	const size_t nn = cp.nodesA.size();
	cp.codeA.assign(3 * nn, 0);
	cp.codeB.assign(3 * nn, 0);
	for (int s = 0; s < 3; s++)
		for (size_t i = 0; i < nn; i++) {
			int a = A.stages[s].outerCode[(size_t)cp.nodesA[i]];
			int b = B.stages[s].outerCode[(size_t)cp.nodesB[i]];
			bool zeroed;
			matchInnersAndOuters(a, b, zeroed);
			cp.codeA[s * nn + i] = (signed char)(a | (zeroed ? 4 : 0));
			cp.codeB[s * nn + i] = (signed char)(b | (zeroed ? 4 : 0));
		}
	// getMaximalPossibleDeterminants (ContactCorrector.hpp:250-276): B along the
	// stage direction, A's LEFT and B's RIGHT outer columns
	if (nn) {
		static const int LEFT[3] = {0, 2, 4}, RIGHT[3] = {1, 3, 5};
		for (int s = 0; s < 3; s++) {
			const double dir[3] = {calc[0][s], calc[1][s], calc[2][s]};
			double B1[3][9], B2[3][9];
			gsx::fixedVelocityGlobal(B1);
			gsx::fixedForceGlobal(dir, B2);
			const double zero[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
			const auto c = gsx::contactCorrection(zero, A.matrices.m[s].U1.data(), LEFT, zero,
			                                      B.matrices.m[s].U1.data(), RIGHT, B1, B2, 0, 0);
			if (!c.ok || !(c.det1 > 0) || !(c.det2 > 0))
				throw Exception("degenerate contact system along the stage direction");
			cp.minDet[s][0] = 1e-3 * c.det1;
			cp.minDet[s][1] = 1e-3 * c.det2;
		}
	}
	return cp;
}

}  // namespace

HostPlans buildHostPlans(const Task& task) {
	if (task.globalSettings.dimensionality != 3) throw Exception("the simplex path is 3-D");
	if (task.bodies.empty()) throw Exception("the simplex task has no bodies");
	// DefaultMesh::applyMaterialsCondition asserts BY_BODIES (engine/simplex/DefaultMesh.hpp:229-230)
	if (task.materialConditions.type != Task::MaterialCondition::Type::BY_BODIES)
		throw Exception("simplex materials must be given BY_BODIES");
	real calc[3][3];
	calcBasis(task, calc);
	const Triangulation tr = buildTriangulation(task);
	HostPlans hp;
	for (const auto& b : task.bodies) hp.bodies.push_back(buildBody(task, tr, b.first, calc));
	// simplex::Engine::estimateTimeStep (Engine.hpp:78-92): minimal over bodies
	hp.tau = std::numeric_limits<real>::max();
	for (const auto& b : hp.bodies) {
		const real t = task.globalSettings.CourantNumber * b.averageHeight / b.maximalEigenvalue;
		if (t < hp.tau) hp.tau = t;
	}
	for (auto& b : hp.bodies) {
		Grid grid(b.mesh);
		for (int s = 0; s < 3; s++) {
			const Real3 dir = {calc[0][s], calc[1][s], calc[2][s]};
			b.stages[s] = buildStagePlan(grid, dir, b.matrices.m[s].L.data(), hp.tau);
		}
		b.border = buildBorderPlan(task, grid, b.matrices, calc, b.stages);
	}
	for (size_t i = 0; i < hp.bodies.size(); i++)  // Utils::makePairs order
		for (size_t j = i + 1; j < hp.bodies.size(); j++)
			hp.contacts.push_back(buildContact(task, tr, hp.bodies, i, j, calc));
	return hp;
}

namespace {
void uploadBody(gsx_ctx* ctx, const BodyPlans& p) {
	std::vector<double> U(3 * 81), U1(3 * 81);
	for (int s = 0; s < 3; s++) {
		std::copy(p.matrices.m[s].U.begin(), p.matrices.m[s].U.end(), U.begin() + s * 81);
		std::copy(p.matrices.m[s].U1.begin(), p.matrices.m[s].U1.end(), U1.begin() + s * 81);
	}
	gcmxCheck(gsx_set_matrices(ctx, U.data(), U1.data()), "gsx_set_matrices");
	const auto& g = p.gradient;
	gcmxCheck(gsx_set_gradient_plan(ctx, g.offsets.data(), g.neighbors.data(), g.rows.data(),
	                                g.weights.data(), g.M.data(), g.det.data()),
	          "gsx_set_gradient_plan");
	for (int s = 0; s < 3; s++) {
		const auto& st = p.stages[s];
		gcmxCheck(gsx_set_stage_plan(ctx, s, st.feet.data(), &st.shift[0][0], (int)st.borderNodes.size(),
		                             st.borderNodes.data(), (int)st.innerNodes.size(),
		                             st.innerNodes.data()),
		          "gsx_set_stage_plan");
	}
	gcmxCheck(gsx_upload(ctx, p.pde.data()), "gsx_upload");
}
}  // namespace

Engine::Engine(const Task& task, int device) : AbstractEngine(task) {
	HostPlans p = buildHostPlans(task);
	tau = p.tau;
	conditions = task.borderConditions;
	for (auto& bp : p.bodies) {
		Body b;
		b.id = bp.id;
		b.materialNumber = task.materialConditions.byBodies.bodyMaterialMap.at(bp.id)->materialNumber;
		const int nv = bp.mesh.nVertices();
		std::vector<double> coords((size_t)nv * 3);
		for (int i = 0; i < nv; i++)
			for (int c = 0; c < 3; c++) coords[(size_t)i * 3 + c] = bp.mesh.v[(size_t)i][c];
		gcmxCheck(gsx_create(device, nv, coords.data(), &b.ctx), "gsx_create");
		bodies.push_back(std::move(b));
		Body& body = bodies.back();
		body.mesh = std::move(bp.mesh);
		uploadBody(body.ctx, bp);
		const auto& bd = bp.border;
		if (!conditions.empty()) {
			gcmxCheck(gsx_set_border_plan(body.ctx, (int)bd.type.size(), bd.type.data(),
			                              bd.minDet.data(), (int)bd.nodes.size(), bd.nodes.data(),
			                              bd.cond.data(), bd.B.data(), bd.S.data(), bd.outer.data()),
			          "gsx_set_border_plan");
			body.hasBorderPlan = true;
		}
	}
	for (const auto& cp : p.contacts) {
		gsx_contact* c = nullptr;
		gcmxCheck(gsx_contact_create(bodies[cp.a].ctx, bodies[cp.b].ctx, (int)cp.nodesA.size(),
		                             cp.nodesA.data(), cp.nodesB.data(), cp.normal.data(), cp.S.data(),
		                             cp.codeA.data(), cp.codeB.data(), &cp.minDet[0][0], &c),
		          "gsx_contact_create");
		contacts.push_back(c);
		contactPairs += cp.nodesA.size();
	}
	// applyPlainBorderContactCorrection(Clock::Time()) (Engine.cpp:44)
	setBorderValues(Clock::Time());
	plainCorrections();
	stepsPerSnap = std::max(1, task.globalSettings.stepsPerSnap);
	for (const Snapshotters::T t : task.globalSettings.snapshottersId) {
		if (t == Snapshotters::T::VTK) vtk = std::make_unique<VtkSnapshotter>(task);
		else throw Exception("only the VTK snapshotter is on the simplex path");
	}
	afterConstruction(task);
}

/// Engine::writeSnapshots (Engine.cpp:313-320) with the VTK snapshotter of every
/// body (VtkSnapshotter.hpp:20-61): the layer is downloaded only when due.
void Engine::writeSnapshots(const int step) {
	if (!vtk || step % stepsPerSnap != 0) return;
	for (size_t i = 0; i < bodies.size(); i++) {
		const std::vector<real> u = pde(i);
		writeVtkSnapshot(vtk->fileName(bodies[i].id, step), bodies[i].mesh.v, bodies[i].mesh.cells,
		                 u.data(), bodies[i].materialNumber, vtk->quantities);
	}
}

void Engine::setBorderValues(real time) {
	std::vector<double> v;
	for (const auto& c : conditions)
		for (const auto& f : c.values) v.push_back(f(time));  // BorderCondition::b (:33-40)
	for (auto& b : bodies)
		if (b.hasBorderPlan) gcmxCheck(gsx_set_border_values(b.ctx, v.data()), "gsx_set_border_values");
}

/// applyPlainBorderContactCorrection (Engine.cpp:193-211): contacts, then borders.
void Engine::plainCorrections() {
	for (auto* c : contacts) gcmxCheck(gsx_contact_plain(c), "gsx_contact_plain");
	for (auto& b : bodies)
		if (b.hasBorderPlan) gcmxCheck(gsx_plain_correction(b.ctx), "gsx_plain_correction");
}

void Engine::setNodeLanes(int lanes) {
	for (auto& b : bodies) gcmxCheck(gsx_set_node_lanes(b.ctx, lanes), "gsx_set_node_lanes");
}

void Engine::setStageFusion(int mode) {
	if (mode < 0) {  // measured per mesh on the next steps (nextTimeStep)
		autoFusion_ = true;
		tunePhase_ = 0;
		mode = 1;
	} else {
		autoFusion_ = false;
	}
	for (auto& b : bodies) gcmxCheck(gsx_set_stage_fusion(b.ctx, mode), "gsx_set_stage_fusion");
	fusionMode_ = mode;
}

long long Engine::launches() const {
	long long n = 0;
	for (const auto& b : bodies) {
		long long k = 0;
		gcmxCheck(gsx_launch_count(b.ctx, &k), "gsx_launch_count");
		n += k;
	}
	return n;
}

Engine::~Engine() {
	for (auto* c : contacts) gsx_contact_destroy(c);
	for (auto& b : bodies) gsx_destroy(b.ctx);
}

real Engine::estimateTimeStep() { return tau; }

// simplex::Engine::nextTimeStep (engine/simplex/Engine.cpp:95-116) with a constant
// basis: plain corrections at the next time layer, then gcmStage (:119-143) for
// every stage: beforeStage + contactAndBorderStage of every body, the contact
// correctors, then (per body) its border correctors, innerStage, afterStage, swap.
// The automatic stage-fusion choice (setStageFusion(-1)) is made on the first
// steps: one warm-up step, kTuneSteps in mode 1, one warm-up step and kTuneSteps
// in mode 2 (with contacts or replayed steps it is not timed: mode 1), each
// block between stream synchronisations; mode 2 is kept only if >= 3 % faster
// (faster on the fracture layer, slower on the cube).  Every
// mode gives the same results (test_one_launch_stage_equals_two_launches), so
// the timed steps are the run's own steps.
void Engine::nextTimeStep() {
	if (autoFusion_ && tunePhase_ < 3 && (!contacts.empty() || replaySteps)) {
		tunePhase_ = 3;  // no timing with contacts or replayed steps: the choice is mode 1
		for (auto& b : bodies) gcmxCheck(gsx_set_stage_fusion(b.ctx, 1), "gsx_set_stage_fusion");
		fusionMode_ = 1;
	}
	const bool tuning = autoFusion_ && tunePhase_ < 3;
	if (tuning && tunePhase_ > 0 && tuneLeft_ == kTuneSteps) {
		sync();
		tuneT0_ = std::chrono::steady_clock::now();
	}
	stepCalls();
	if (!tuning) return;
	if (tunePhase_ == 0) {
		tunePhase_ = 1;
		tuneLeft_ = kTuneSteps;
		return;
	}
	if (--tuneLeft_ > 0) return;
	sync();
	tuneMs_[tunePhase_ - 1] =
	    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tuneT0_).count() / kTuneSteps;
	if (tunePhase_ == 1) {
		tunePhase_ = 2;
		tuneLeft_ = kTuneSteps + 1;  // one untimed step in mode 2 first (its first-use costs)
		for (auto& b : bodies) gcmxCheck(gsx_set_stage_fusion(b.ctx, 2), "gsx_set_stage_fusion");
		fusionMode_ = 2;
	} else {
		tunePhase_ = 3;
		const int best = tuneMs_[1] < 0.97 * tuneMs_[0] ? 2 : 1;
		for (auto& b : bodies) gcmxCheck(gsx_set_stage_fusion(b.ctx, best), "gsx_set_stage_fusion");
		fusionMode_ = best;
	}
}

void Engine::stepCalls() {
	setBorderValues(Clock::Time() + Clock::TimeStep());
	if (replaySteps) {  // the same calls, captured once per layer state and replayed
		std::vector<gsx_ctx*> ctxs;
		for (auto& b : bodies) ctxs.push_back(b.ctx);
		gcmxCheck(gsx_step(ctxs.data(), (int)ctxs.size(), contacts.data(), (int)contacts.size()),
		          "gsx_step");
		return;
	}
	plainCorrections();
	for (int stage = 0; stage < 3; stage++) {
		if (contacts.empty()) {  // nothing between a body's halves: gsx_stage may run them as one launch
			for (auto& b : bodies) {
				gcmxCheck(gsx_stage(b.ctx, stage), "gsx_stage");
				int fused = 0;
				gcmxCheck(gsx_last_stage_fused(b.ctx, &fused), "gsx_last_stage_fused");
				fusedStages_ += fused;
			}
			continue;
		}
		for (auto& b : bodies) gcmxCheck(gsx_stage_nodes(b.ctx, stage), "gsx_stage_nodes");
		for (auto* c : contacts) gcmxCheck(gsx_contact_correct(c, stage), "gsx_contact_correct");
		for (auto& b : bodies) gcmxCheck(gsx_stage_finish(b.ctx, stage), "gsx_stage_finish");
	}
}

void Engine::sync() const {
	for (const auto& b : bodies) gcmxCheck(gsx_sync(b.ctx), "gsx_sync");
}

std::pair<bool, int> Engine::stagePlanInfo(size_t body, int stage) const {
	int fusable = 0, waits = 0;
	gcmxCheck(gsx_stage_plan_info(bodies.at(body).ctx, stage, &fusable, &waits), "gsx_stage_plan_info");
	return {fusable != 0, waits};
}

void Engine::setWaitBudget(int polls) {
	for (auto& b : bodies) gcmxCheck(gsx_set_wait_budget(b.ctx, polls), "gsx_set_wait_budget");
}

size_t Engine::numberOfContactPairs() const { return contactPairs; }

std::vector<real> Engine::pde(size_t body) const {
	const Body& b = bodies.at(body);
	std::vector<real> out((size_t)b.mesh.nVertices() * 9);
	gcmxCheck(gsx_download(b.ctx, out.data()), "gsx_download");
	return out;
}

}  // namespace simplex
}  // namespace gcm
