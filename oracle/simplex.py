"""CPU oracle for the simplex (tetrahedral) grid-characteristic path.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.py for the rules: only tests/,
``__graft_entry__.smoke()`` and bench.py's cpu_baseline may import this).

A plain-Python restatement of the reference's simplex stage in Riemann
invariants for one isotropic-elastic body with a constant calculation basis,
GLOBAL_BASIS border mode, PRODUCT splitting and the border correctors of
Task::borderConditions (FIXED_FORCE / FIXED_VELOCITY; border nodes no condition
covers keep zero outer invariants):

* triangulation queries over a given tetrahedral mesh (the mesh is INPUT: CGAL,
  the reference's mesher, is absent; tests take the product's boxMesh output as
  the task's mesh, like a mesh file): incident cells in ascending cell order,
  face neighbours, the line walk of grid/simplex/cgal/LineWalker.hpp:25-88 and
  SimplexGrid::findCellCrossedByTheRay (grid/simplex/SimplexGrid.cpp:57-164);
* Differentiation::estimateGradient (util/math/Differentiation.hpp:33-63);
* GridCharacteristicMethodInRiemannInvariants (engine/simplex/
  GridCharacteristicMethodInRiemannInvariants.hpp:44-198) with
  TetrahedronInterpolator::hybridInterpolate / interpolateInOwner
  (util/math/interpolation/TetrahedronInterpolator.hpp:93-155) and
  interpolateInSpaceTime (engine/simplex/common.hpp:102-129);
* BorderCorrectorInRiemannInvariants / BorderCorrectorInPdeVectors
  (engine/simplex/BorderCorrector.hpp:82-276), calculateOuterWaveCorrection
  (common.hpp:153-202), ElasticModel::borderMatrixFixedForce / FixedVelocity /
  applyPlainBorderCorrection (rheology/models/ElasticModel.hpp:111-228), border
  node selection (Engine::addBorderNode, Engine.cpp:292-309) with
  SimplexGrid::normal (grid/simplex/SimplexGrid.hpp:426-444);
* simplex::Engine::nextTimeStep / gcmStage (engine/simplex/Engine.cpp:95-135).

Every expression keeps the reference's operation order on Python floats (IEEE
double), so results are bit-for-bit comparable.  Parity against the reference
itself is UNPINNED: CGAL is absent, so neither the reference's meshes nor its
simplex outputs can be produced here; the only in-repo pins are structural
(TestSimplexGcm.cpp:29-67, zero state stays zero), checked in tests.
Paths are relative to /root/reference/src/libgcm.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

EQUALITY_TOLERANCE = 1e-9   # util/infrastructure/Types.hpp:10
MAX_NB = 20                 # Cgal3DTriangulation.hpp:53
RIGHT = [1, 3, 5]           # rheology/models/Model.cpp:81-82
LEFT = [0, 2, 4]


# -------------------------------------------------------------- linal --

def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def _mul(a, x):
    return (a[0] * x, a[1] * x, a[2] * x)


def _dot(a, b):  # linal/functions.hpp:327-334
    r = a[0] * b[0]
    r += a[1] * b[1]
    r += a[2] * b[2]
    return r


def _length(a):
    return math.sqrt(_dot(a, a))


def _cross(a, b):  # linal/geometry.hpp:13-17
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def _det3(m11, m12, m13, m21, m22, m23, m31, m32, m33):  # linal/determinants.hpp:40-53
    return m11 * (m22 * m33 - m23 * m32) - m12 * (m21 * m33 - m23 * m31) + \
        m13 * (m21 * m32 - m22 * m31)


def _det2(m11, m12, m21, m22):
    return m11 * m22 - m12 * m21


def _solve3(A, b):  # linal/linearSystems.hpp:104-129
    det = _det3(A[0][0], A[0][1], A[0][2], A[1][0], A[1][1], A[1][2], A[2][0], A[2][1], A[2][2])
    if det == 0:
        raise ValueError("SLE determinant is zero")
    d1 = _det3(b[0], A[0][1], A[0][2], b[1], A[1][1], A[1][2], b[2], A[2][1], A[2][2])
    d2 = _det3(A[0][0], b[0], A[0][2], A[1][0], b[1], A[1][2], A[2][0], b[2], A[2][2])
    d3 = _det3(A[0][0], A[0][1], b[0], A[1][0], A[1][1], b[1], A[2][0], A[2][1], b[2])
    return (d1 / det, d2 / det, d3 / det)


def _tmul_cols(cols, b):
    """transposeMultiply(A, b) for A given by columns (functions.hpp:220-234)."""
    out = []
    for c in cols:
        s = c[0] * b[0]
        for n in range(1, len(b)):
            s += c[n] * b[n]
        out.append(s)
    return out


def _lls32(c0, c1, b):  # linearLeastSquares 3x2, W = I (linearSystems.hpp:150-158)
    cols = [c0, c1]
    M = [[_tmul_cols([ci], cj)[0] for cj in cols] for ci in cols]
    r = _tmul_cols(cols, b)
    det = _det2(M[0][0], M[0][1], M[1][0], M[1][1])
    if det == 0:
        raise ValueError("SLE determinant is zero")
    return (_det2(r[0], M[0][1], r[1], M[1][1]) / det, _det2(M[0][0], r[0], M[1][0], r[1]) / det)


def _lls31(c0, b):
    m = _tmul_cols([c0], c0)[0]
    r = _tmul_cols([c0], b)[0]
    if m == 0:
        raise ValueError("SLE determinant is zero")
    return r / m


def barycentric4(a, b, c, d, q):  # geometry.hpp:142-151
    T = [[a[0] - d[0], b[0] - d[0], c[0] - d[0]],
         [a[1] - d[1], b[1] - d[1], c[1] - d[1]],
         [a[2] - d[2], b[2] - d[2], c[2] - d[2]]]
    l = _solve3(T, _sub(q, d))
    return (l[0], l[1], l[2], 1 - l[0] - l[1] - l[2])


# ---- TetrahedronInterpolator / TriangleInterpolator (util/math/interpolation/
# TetrahedronInterpolator.hpp, TriangleInterpolator.hpp) as standalone functions:
# the reference's own known answers (src/test/sequence/TestInterpolator.cpp:
# 129-282) pin them (tests/test_simplex_cpu.py); _interp below uses the same ones.
_TET_TRIES = [(0, 1, 2, 3), (0, 1, 2, 4), (0, 1, 2, 5), (0, 1, 3, 4), (0, 1, 3, 5), (0, 1, 4, 5),
              (0, 2, 3, 4), (0, 2, 3, 5), (0, 2, 4, 5), (0, 3, 4, 5), (1, 2, 3, 4), (1, 2, 3, 5),
              (1, 2, 4, 5), (1, 3, 4, 5), (2, 3, 4, 5)]


def _is_interpolation(lam):  # TetrahedronInterpolator.hpp:15-20 / TriangleInterpolator.hpp:15-19
    return all(l > -EQUALITY_TOLERANCE for l in lam)


def tet_weights(c, q):
    """barycentricCoordinates + the isInterpolation assert (hpp:33-34)."""
    lam = barycentric4(c[0], c[1], c[2], c[3], q)
    if not _is_interpolation(lam):
        raise ValueError("isInterpolation")  # assert_true throws gcm::Exception
    return lam


def tet_linear_lam(lam, v):  # hpp:35-38: lambda(0) * v0 + ... + lambda(3) * v3
    return lam[0] * v[0] + lam[1] * v[1] + lam[2] * v[2] + lam[3] * v[3]


def tet_quadratic_lam(lam, c, v, g, q):  # hpp:54-58
    t = [v[i] + _dot(g[i], _sub(q, c[i])) / 2.0 for i in range(4)]
    return lam[0] * t[0] + lam[1] * t[1] + lam[2] * t[2] + lam[3] * t[3]


def _limiter_min_max(u, vals):  # linal/functions.hpp:676-679: min(max(u, min(vals)), max(vals))
    mn, mx = vals[0], vals[0]
    for x in vals[1:]:
        mn, mx = _std_min(mn, x), _std_max(mx, x)
    return _std_min(_std_max(u, mn), mx)


def tet_linear(c, v, q):  # TetrahedronInterpolator::interpolate, linear (hpp:27-38)
    return tet_linear_lam(tet_weights(c, q), v)


def tet_quadratic(c, v, g, q):  # TetrahedronInterpolator::interpolate, quadratic (hpp:47-58)
    return tet_quadratic_lam(tet_weights(c, q), c, v, g, q)


def tet_min_max(c, v, g, q):  # minMaxInterpolate (hpp:69-78)
    return _limiter_min_max(tet_quadratic(c, v, g, q), v)


def tet_hybrid_lam(lam, c, v, g, q):  # hybridInterpolate (hpp:93-104) with the weights given
    quad = tet_quadratic_lam(lam, c, v, g, q)
    return quad if quad == _limiter_min_max(quad, v) else tet_linear_lam(lam, v)


def tet_hybrid(c, v, g, q):
    return tet_hybrid_lam(tet_weights(c, q), c, v, g, q)


def tet_owner_pick(c6, q):
    """interpolateInOwner's choice (hpp:113-155): (point indices, barycentrics)."""
    for tr in _TET_TRIES:
        if _volume(*[c6[i] for i in tr]) != 0:
            lam = barycentric4(*[c6[i] for i in tr], q)
            if _is_interpolation(lam):
                return tr, lam
    raise ValueError("Containing tetrahedron is not found")


def tet_interpolate_in_owner(c6, v6, q):
    tr, lam = tet_owner_pick(c6, q)
    return tet_linear_lam(lam, [v6[i] for i in tr])


def tri_barycentric(a, b, c, q):  # geometry.hpp:108-116 (2-D): 2x2 Cramer (linearSystems.hpp:71-90)
    T = [[a[0] - c[0], b[0] - c[0]], [a[1] - c[1], b[1] - c[1]]]
    r = (q[0] - c[0], q[1] - c[1])
    det = _det2(T[0][0], T[0][1], T[1][0], T[1][1])
    if det == 0:
        raise ValueError("SLE determinant is zero")
    l0 = _det2(r[0], T[0][1], r[1], T[1][1]) / det
    l1 = _det2(T[0][0], r[0], T[1][0], r[1]) / det
    return (l0, l1, 1 - l0 - l1)


def tri_weights(a, b, c, q):  # + the isInterpolation assert (TriangleInterpolator.hpp:32-33)
    lam = tri_barycentric(a, b, c, q)
    if not _is_interpolation(lam):
        raise ValueError("isInterpolation")
    return lam


def tri_linear(c, v, q):  # TriangleInterpolator::interpolate, linear (hpp:26-36)
    lam = tri_weights(c[0], c[1], c[2], q)
    return lam[0] * v[0] + lam[1] * v[1] + lam[2] * v[2]


def tri_quadratic(c, v, g, q):  # TriangleInterpolator::interpolate, quadratic (hpp:45-56)
    lam = tri_weights(c[0], c[1], c[2], q)
    t = [v[i] + (g[i][0] * (q[0] - c[i][0]) + g[i][1] * (q[1] - c[i][1])) / 2.0 for i in range(3)]
    return lam[0] * t[0] + lam[1] * t[1] + lam[2] * t[2]


def tri_min_max(c, v, g, q):  # TriangleInterpolator::minMaxInterpolate
    return _limiter_min_max(tri_quadratic(c, v, g, q), v)


def tri_interpolate_in_owner(c4, v4, q):  # TriangleInterpolator::interpolateInOwner (TRY_TRIANGLE order)
    for tr in [(0, 1, 2), (0, 1, 3), (0, 2, 3), (1, 2, 3)]:
        lam = tri_barycentric(*[c4[i] for i in tr], q)  # a zero determinant throws, as in the reference
        if _is_interpolation(lam):
            return lam[0] * v4[tr[0]] + lam[1] * v4[tr[1]] + lam[2] * v4[tr[2]]
    raise ValueError("Containing triangle is not found")


def _barycentric3(a, b, c, q):  # geometry.hpp:124-137
    l = _lls32(_sub(a, c), _sub(b, c), _sub(q, c))
    return (l[0], l[1], 1 - l[0] - l[1])


def _barycentric2(a, b, q):  # geometry.hpp:88-103
    l = _lls31(_sub(a, b), _sub(q, b))
    return (l, 1 - l)


def oriented_volume(a, b, c, d):  # geometry.hpp:248-255
    ba, ca, da = _sub(b, a), _sub(c, a), _sub(d, a)
    return _det3(ba[0], ba[1], ba[2], ca[0], ca[1], ca[2], da[0], da[1], da[2]) / 6


def _volume(a, b, c, d):
    return abs(oriented_volume(a, b, c, d))


def _area(a, b, c):
    return _length(_cross(_sub(b, a), _sub(c, a))) / 2


def _min_height3(a, b, c):
    S = _area(a, b, c)
    ab, ac, bc = _length(_sub(a, b)), _length(_sub(a, c)), _length(_sub(b, c))
    return 2 * S / max(ab, max(ac, bc))


def min_height4(a, b, c, d):  # geometry.hpp:274-284
    V = _volume(a, b, c, d)
    A, B, C, D = _area(b, c, d), _area(c, d, a), _area(d, a, b), _area(a, b, c)
    return 3 * V / max(A, max(B, max(C, D)))


def _degenerate3(a, b, c, eps):
    h = _min_height3(a, b, c)
    l = (_length(_sub(a, b)) + _length(_sub(a, c)) + _length(_sub(b, c))) / 3
    return h <= eps * l


def _degenerate4(a, b, c, d, eps):
    h = min_height4(a, b, c, d)
    l = (_length(_sub(a, b)) + _length(_sub(a, c)) + _length(_sub(a, d)) + _length(_sub(d, b)) +
         _length(_sub(d, c)) + _length(_sub(b, c))) / 6
    return h <= eps * l


def _segment_contains(a, b, q, eps, deg):
    if not _degenerate3(a, b, q, deg):
        return False
    l = _barycentric2(a, b, q)
    return l[0] >= -eps and l[1] >= -eps


def _triangle_contains(a, b, c, q, eps, deg):
    if not _degenerate4(a, b, c, q, deg):
        return False
    l = _barycentric3(a, b, c, q)
    return l[0] >= -eps and l[1] >= -eps and l[2] >= -eps


def _tet_contains(a, b, c, d, q, eps):
    l = barycentric4(a, b, c, d, q)
    return l[0] >= -eps and l[1] >= -eps and l[2] >= -eps and l[3] >= -eps


def _solid_angle_contains(a, b, c, d, q, eps):
    l = barycentric4(a, b, c, d, q)
    return l[0] <= 1 + eps and l[1] >= -eps and l[2] >= -eps and l[3] >= -eps


def _line_flat(f1, f2, f3, l1, l2):  # geometry.hpp:201-217
    tau, p, q = _sub(l2, l1), _sub(f2, f1), _sub(f3, f1)
    A = [[tau[0], -p[0], -q[0]], [tau[1], -p[1], -q[1]], [tau[2], -p[2], -q[2]]]
    params = _solve3(A, _sub(f1, l1))
    return _add(l1, _mul(tau, params[0]))


def _neg(a):
    return (-a[0], -a[1], -a[2])


def _normalize(a):  # linal/functions.hpp:375-379
    l = _length(a)
    return (a[0] / l, a[1] / l, a[2] / l)


def _opposite_face_normal(opposite, a, b, c):  # geometry.hpp:423-428
    ans = _normalize(_cross(_sub(a, b), _sub(c, b)))
    return ans if _dot(ans, _sub(a, opposite)) > 0 else _neg(ans)


def local_basis(n):  # linal/basis.hpp:59-65, perpendicularClockwise geometry.hpp:46-52
    """Rows of the 3x3 matrix with columns (tau1, tau2, n)."""
    ans = (n[1], -n[0], 0.0)
    if n[0] == 0 and n[1] == 0:
        ans = (n[2], 0.0, 0.0)
    lv, la = _length(n), _length(ans)
    t1 = tuple((x * lv) / la for x in ans)
    t2 = _cross(n, t1)
    return [[t1[r], t2[r], n[r]] for r in range(3)]


def _sym(i, j):  # linal/Symmetry.hpp:38-46 + VelocitySigmaVariables.hpp:82-96
    a, b = min(i, j), max(i, j)
    return 3 + a * 3 - ((a - 1) * a) // 2 + b - a


def border_matrix(kind, normal):  # ElasticModel.hpp:111-154, 3 x 9
    S = local_basis(normal)
    B = [[0.0] * 9 for _ in range(3)]
    if kind == "FIXED_FORCE":
        for k in range(3):
            G = [0.0] * 6          # SymmetricMatrix::Zeros; (i, j) and (j, i) share a slot
            for i in range(3):
                for j in range(3):
                    q = _sym(i, j) - 3
                    G[q] = G[q] + S[i][k] * normal[j]
            for q in range(6):
                B[k][3 + q] = G[q]  # setSigma
    elif kind == "FIXED_VELOCITY":
        for i in range(3):
            for j in range(3):
                B[i][j] = S[j][i]   # setVelocity(S.getColumn(i))
    else:
        raise ValueError("Unknown type of border condition")
    return B


def _mat_mul(A, B):  # linal/operators.hpp:98-123
    n, m, k = len(A), len(B), len(B[0])
    out = []
    for i in range(n):
        row = []
        for j in range(k):
            x = A[i][0] * B[0][j]
            for t in range(1, m):
                x += A[i][t] * B[t][j]
            row.append(x)
        out.append(row)
    return out


def _det33(M):
    return _det3(M[0][0], M[0][1], M[0][2], M[1][0], M[1][1], M[1][2], M[2][0], M[2][1], M[2][2])


def outer_wave_correction(u, Omega, B, b, min_valid):  # common.hpp:186-202
    """(determinant fabs, successful, value) -- Omega: 9 x 3, B: 3 x 9."""
    M = _mat_mul(B, Omega)
    det = abs(_det33(M))
    if not det > min_valid:
        return det, False, [0.0] * 9
    Bu = _mat_mul(B, [[x] for x in u])
    rhs = [b[i] - Bu[i][0] for i in range(3)]
    alpha = _solve3(M, rhs)
    value = _mat_mul(Omega, [[a] for a in alpha])
    return det, True, [v[0] for v in value]


def plain_border_correction(u, kind, normal, value):  # ElasticModel.hpp:202-228
    u = list(u)
    S = local_basis(normal)
    if kind == "FIXED_FORCE":
        sg = [[u[_sym(i, j)] for j in range(3)] for i in range(3)]   # getSigmaFrom
        ST = [[S[j][i] for j in range(3)] for i in range(3)]
        sl = _mat_mul(_mat_mul(ST, sg), S)
        for i in range(3):
            sl[i][2] = value[i]     # setColumn(D - 1)
        for j in range(3):
            sl[2][j] = value[j]     # setRow(D - 1)
        sg = _mat_mul(_mat_mul(S, sl), ST)
        for i in range(3):
            for j in range(3):
                u[_sym(i, j)] = sg[i][j]   # setSigmaTo: row-major, the later write wins
    else:
        v = _mat_mul(S, [[x] for x in value])
        for i in range(3):
            u[i] = v[i][0]
    return u


# --------------------------------------------------------------- grid --

EMPTY = -1                  # Grid::EmptySpaceFlag


class Grid:
    """SimplexGrid<3> over a given mesh (coords [n][3], cells [m][4]).  For a body of
    a multi-body task, ``face_grid(cell, i)`` names the grid across a face with no
    neighbour in the body (EMPTY or another body id) and ``other_grids[it]`` the
    other grid ids around a vertex (SimplexGrid::gridsAroundVertex minus its own)."""

    def __init__(self, coords: Sequence[Sequence[float]], cells: Sequence[Sequence[int]],
                 face_grid=None, other_grids=None):
        self.P = [tuple(float(x) for x in c) for c in coords]
        self.cells = [tuple(int(x) for x in c) for c in cells]
        nv = len(self.P)
        faces = {}
        self.nb = [[-1] * 4 for _ in self.cells]
        for ci, c in enumerate(self.cells):
            for i in range(4):
                f = tuple(sorted((c[(i + 1) % 4], c[(i + 2) % 4], c[(i + 3) % 4])))
                if f in faces:
                    cj, j = faces.pop(f)
                    self.nb[ci][i] = cj
                    self.nb[cj][j] = ci
                else:
                    faces[f] = (ci, i)
        self.inc = [[] for _ in range(nv)]
        for ci, c in enumerate(self.cells):
            for x in c:
                self.inc[x].append(ci)
        self.inner = [True] * nv
        for ci, c in enumerate(self.cells):
            for i in range(4):
                if self.nb[ci][i] < 0:
                    for k in range(1, 4):
                        self.inner[c[(i + k) % 4]] = False
        self.face_grid = face_grid or (lambda ci, i: EMPTY)
        if other_grids is None:
            other_grids = [[] if self.inner[i] else [EMPTY] for i in range(nv)]
        self.other_grids = other_grids
        for i in range(nv):
            assert (not other_grids[i]) == self.inner[i]
        # markInnersAndBorders (SimplexGrid.cpp:216-252)
        self.inner_idx = [i for i in range(nv) if self.inner[i]]
        self.contact_idx = [i for i in range(nv) if len(other_grids[i]) == 1
                            and other_grids[i][0] != EMPTY]
        cs = set(self.contact_idx)
        self.border_idx = [i for i in range(nv) if not self.inner[i] and i not in cs]
        self.average_height = self._average_height()

    def border_normal(self, it):  # SimplexGrid.hpp:151-154, 426-444; Cgal3DTriangulation.hpp:109-118
        return self.normal(it, lambda g: g == EMPTY)

    def contact_normal(self, it, other):  # SimplexGrid.hpp:141-144
        return self.normal(it, lambda g: g == other)

    def common_normal(self, it):  # SimplexGrid.hpp:157-160
        return self.normal(it, lambda g: True)

    def normal(self, it, use):
        normals = []
        for ci in self.inc[it]:
            c = self.cells[ci]
            for i in range(4):
                if self.nb[ci][i] < 0 and c[i] != it and use(self.face_grid(ci, i)):
                    normals.append(_opposite_face_normal(
                        self.P[c[i]], self.P[c[(i + 1) % 4]], self.P[c[(i + 2) % 4]],
                        self.P[c[(i + 3) % 4]]))
        if not normals:
            return (0.0, 0.0, 0.0)
        acc = (0.0, 0.0, 0.0)
        for n in normals:
            acc = _add(acc, n)
        return _normalize(acc)

    def _average_height(self):  # SimplexGrid.cpp:266-285 + util/math/Histogram.hpp
        hs = [min_height4(*[self.P[x] for x in c]) for c in self.cells]
        mn, mx = min(hs), max(hs)
        nbins = 100
        bs0 = (mx - mn) / float(nbins)
        if mx == mn:
            bins = [0] * nbins
            bins[0] = len(hs)
        else:
            bins = [0] * (nbins + 1)
            for h in hs:
                bins[int((h - mn) / bs0)] += 1
            bins[nbins - 1] += bins[-1]
            bins.pop()
        bs = (mx - mn) / float(len(bins))
        ip, cnt = 0.0, 0.0
        for i, b in enumerate(bins):
            ip = ip + float(b) * (mn + (float(i) + 0.5) * bs)
            cnt = cnt + float(b)
        return ip / cnt

    def neighbors(self, it) -> List[int]:  # SimplexGrid.hpp:249-259
        s = set()
        for c in self.inc[it]:
            s.update(self.cells[c])
        s.discard(it)
        return sorted(s)

    def _other_index(self, cell, a, b, c):
        for i in range(4):
            d = self.cells[cell][i]
            if d != a and d != b and d != c:
                return i
        raise ValueError("Cell contains equal vertices")

    def _crossed_incident(self, vh, query, eps):  # Cgal3DTriangulation.hpp:221-238
        for cand in self.inc[vh]:
            t = self.cells[cand]
            a = t[self._other_index(cand, vh, vh, vh)]
            b = t[self._other_index(cand, vh, vh, a)]
            c = t[self._other_index(cand, vh, a, b)]
            if _solid_angle_contains(self.P[vh], self.P[a], self.P[b], self.P[c], query, eps):
                return cand
        return -1

    def _inside_out_facet(self, t, q, p, eps):  # Cgal3DTriangulation.hpp:247-259
        for i in range(4):
            a, b, c = (self.cells[t][(i + k) % 4] for k in (1, 2, 3))
            if _solid_angle_contains(q, self.P[a], self.P[b], self.P[c], p, eps):
                return a, b, c
        return None

    def _collect(self, q, p, t, u, v, w):  # LineWalker.hpp:25-52
        P = self.P
        ans, last_face = [t], None
        while oriented_volume(P[u], P[v], P[w], p) < 0:
            nt = self.nb[t][self._other_index(t, u, v, w)]
            if nt < 0:
                ans.append(-1)
                last_face = (u, v, w)
                break
            t = nt
            ans.append(t)
            s = self.cells[t][self._other_index(t, u, v, w)]
            if oriented_volume(P[u], P[s], q, p) > 0:
                if oriented_volume(P[v], P[s], q, p) > 0:
                    u = s
                else:
                    w = s
            else:
                if oriented_volume(P[w], P[s], q, p) > 0:
                    v = s
                else:
                    u = s
        return ans, last_face

    def _along_from_vertex(self, q, p):  # LineWalker.hpp:54-69
        t = self._crossed_incident(q, p, 0.0)
        if t < 0:
            return [], None
        c = self.cells[t]
        u = c[self._other_index(t, q, q, q)]
        v = c[self._other_index(t, q, q, u)]
        w = c[self._other_index(t, q, u, v)]
        if oriented_volume(self.P[u], self.P[v], self.P[w], self.P[q]) < 0:
            u, v = v, u
        return self._collect(self.P[q], p, t, u, v, w)

    def _along_from_cell(self, t, q, p):  # LineWalker.hpp:71-88
        f = self._inside_out_facet(t, q, p, 0.0)
        if f is None:
            f = self._inside_out_facet(t, q, p, EQUALITY_TOLERANCE)
        if f is None:
            return [], None
        u, v, w = f
        if oriented_volume(self.P[u], self.P[v], self.P[w], q) < 0:
            u, v = v, u
        return self._collect(q, p, t, u, v, w)

    def _contains(self, c, q):
        return _tet_contains(*[self.P[x] for x in self.cells[c]], q, EQUALITY_TOLERANCE)

    def _check(self, it, along, last_face, start, query):  # SimplexGrid.cpp:115-164
        if not along:
            return []
        last = along[-1]
        if last >= 0 and self._contains(last, query):
            return list(self.cells[last])
        if len(along) == 1:
            if self.inner[it]:
                raise ValueError("one-cell walk from an inner node")
            return []
        prev = along[-2]
        if self._contains(prev, query):
            return list(self.cells[prev])
        if not self.inner[it]:
            return []
        if last < 0:
            face = [x for x in self.cells[prev] if x in last_face]
            p = [self.P[x] for x in face]
            x = _line_flat(p[0], p[1], p[2], start, query)
            if _triangle_contains(p[0], p[1], p[2], x, EQUALITY_TOLERANCE, EQUALITY_TOLERANCE):
                return face
            for i in range(3):
                for j in range(i + 1, 3):
                    if _segment_contains(p[i], p[j], x, EQUALITY_TOLERANCE, EQUALITY_TOLERANCE):
                        return [face[i], face[j]]
            for i in range(3):
                if _segment_contains(start, query, p[i], EQUALITY_TOLERANCE, EQUALITY_TOLERANCE):
                    return [face[i]]
            return []
        return []

    def find_cell(self, it, shift) -> List[int]:  # SimplexGrid.cpp:57-112
        start = self.P[it]
        query = _add(start, shift)
        along, lf = self._along_from_vertex(it, query)
        found = self._check(it, along, lf, start, query)
        if found:
            return found
        sc = self._crossed_incident(it, query, 0.0)
        if sc < 0:
            sc = self._crossed_incident(it, query, EQUALITY_TOLERANCE)
        if sc < 0:
            sc = self.inc[it][0]
        t = [self.P[x] for x in self.cells[sc]]
        cen = _add(_add(_add(t[0], t[1]), t[2]), t[3])
        cen = (cen[0] / 4, cen[1] / 4, cen[2] / 4)
        w = 1e-3
        start_point = _add(_mul(cen, w), _mul(start, 1 - w))
        along, lf = self._along_from_cell(sc, start_point, query)
        found = self._check(it, along, lf, start, query)
        if found:
            return found
        if self.inner[it]:
            raise ValueError("line walk failed for an inner node")
        return []

    # -- Differentiation::estimateGradient -----------------------------------
    def gradients(self, w: List[List[float]]):
        """w[node][k] -> grad[node][r][k] (Differentiation.hpp:33-63)."""
        out = []
        for it in range(len(self.P)):
            nbs = self.neighbors(it)[:MAX_NB]
            A = [[0.0] * 3 for _ in range(MAX_NB)]
            W = [0.0] * MAX_NB
            b = [[0.0] * 9 for _ in range(MAX_NB)]
            for i, nb in enumerate(nbs):
                d = _sub(self.P[nb], self.P[it])
                A[i] = list(d)
                W[i] = 1.0 / _length(d)
                b[i] = [w[nb][k] - w[it][k] for k in range(9)]
            WA = [[W[i] * A[i][c] for c in range(3)] for i in range(MAX_NB)]
            M = [[None] * 3 for _ in range(3)]
            for r in range(3):
                for c in range(3):
                    s = A[0][r] * WA[0][c]
                    for n in range(1, MAX_NB):
                        s += A[n][r] * WA[n][c]
                    M[r][c] = s
            g = [[0.0] * 9 for _ in range(3)]
            for k in range(9):
                Wb = [b[i][k] * W[i] for i in range(MAX_NB)]
                rhs = []
                for r in range(3):
                    s = A[0][r] * Wb[0]
                    for n in range(1, MAX_NB):
                        s += A[n][r] * Wb[n]
                    rhs.append(s)
                x = _solve3(M, rhs)
                for r in range(3):
                    g[r][k] = x[r]
            out.append(g)
        return out


def _std_min(a, b):
    return b if b < a else a


def _std_max(a, b):
    return b if a < b else a


class Engine:
    """simplex::Engine<3> for one body (see module docstring)."""

    def __init__(self, coords, cells, U, U1, L, basis, courant, pde0, border_conditions=(),
                 grid=None, tau=None):
        """U, U1: [3][9][9]; L: [3][9]; basis: 3x3 (column s = stage s); pde0 [n][9];
        border_conditions: Task::borderConditions as dicts {"contains": point -> bool,
        "type": "FIXED_FORCE" | "FIXED_VELOCITY", "values": [3 functions of t],
        "multi": useForMulticontactNodes}."""
        self.grid = grid if grid is not None else Grid(coords, cells)
        self.U = [[[float(x) for x in row] for row in U[s]] for s in range(3)]
        self.U1 = [[[float(x) for x in row] for row in U1[s]] for s in range(3)]
        self.L = [[float(x) for x in L[s]] for s in range(3)]
        self.basis = [[float(basis[r][c]) for c in range(3)] for r in range(3)]
        mx = 0.0
        for s in range(3):
            for k in range(9):
                mx = max(mx, abs(self.L[s][k]))
        self.tau = courant * self.grid.average_height / mx  # Engine.hpp:78-92
        if tau is not None:
            self.tau = tau                    # minimal over the bodies
        self.u = [[float(x) for x in row] for row in pde0]
        self.outers = [{} for _ in range(3)]
        self.feet = [self._plan(s) for s in range(3)]
        self.time = 0.0
        self.conditions = list(border_conditions)
        self._border_setup()
        self._plain_correction(self.time)     # Engine.cpp:44

    def _border_setup(self):
        """Engine::createMeshes' Border list + addBorderNode (Engine.cpp:76-84, 292-309)."""
        g = self.grid
        self.corrected = []                   # (node, condition, normal)
        for it in g.border_idx:
            multi = g.border_normal(it) == (0.0, 0.0, 0.0)
            chosen = None
            for ci, c in enumerate(self.conditions):
                if c["contains"](g.P[it]) and (not multi or c.get("multi", True)):
                    chosen = ci
            if chosen is None:
                continue
            n = g.common_normal(it)
            if n == (0.0, 0.0, 0.0):
                raise ValueError("zero common normal at a border node")
            self.corrected.append((it, chosen, n))
        self.min_det = {}
        for ci, c in enumerate(self.conditions):   # getMaximalPossibleDeterminant (hpp:198-214)
            if not any(x[1] == ci for x in self.corrected):
                continue
            for s in range(3):
                direction = (self.basis[0][s], self.basis[1][s], self.basis[2][s])
                det, ok, _ = outer_wave_correction([0.0] * 9, self._omega(s, RIGHT),
                                                   border_matrix(c["type"], direction), [0.0] * 3, 0)
                if not (ok and det > 0):
                    raise ValueError("degenerate outer-wave system")
                self.min_det[(ci, s)] = 1e-3 * det

    def _omega(self, s, cols):  # getColumnsFromGcmMatrices (common.hpp:153-165)
        return [[self.U1[s][i][c] for c in cols] for i in range(9)]

    def _b(self, ci, t):
        return [float(f(t)) for f in self.conditions[ci]["values"]]

    def _plain_correction(self, t):  # applyPlainBorderContactCorrection (Engine.cpp:193-211)
        for it, ci, n in self.corrected:
            self.u[it] = plain_border_correction(self.u[it], self.conditions[ci]["type"], n,
                                                 self._b(ci, t))

    def _correct(self, s, wn, t):
        """BorderCorrectorInRiemannInvariants::applyInGlobalBasis (hpp:256-265)."""
        for it, ci, n in self.corrected:
            kind = self.conditions[ci]["type"]
            b = self._b(ci, t)
            min_valid = self.min_det[(ci, s)]
            B = border_matrix(kind, n)
            u = self._mat_vec(self.U1[s], wn[it])
            outers = self.outers[s].get(it, [])
            if outers == RIGHT or outers == LEFT:
                _, ok, v = outer_wave_correction(u, self._omega(s, outers), B, b, min_valid)
                if ok:
                    u = [u[i] + v[i] for i in range(9)]
                else:
                    u = plain_border_correction(u, kind, n, b)
            else:
                _, okr, vr = outer_wave_correction(u, self._omega(s, RIGHT), B, b, min_valid)
                _, okl, vl = outer_wave_correction(u, self._omega(s, LEFT), B, b, min_valid)
                if okr and okl:
                    u = [u[i] + (vr[i] + vl[i]) / 2 for i in range(9)]
                else:
                    u = plain_border_correction(u, kind, n, b)
            wn[it] = self._mat_vec(self.U[s], u)

    def _plan(self, s):
        """Per node and invariant 0..5: ('cell', verts, q) | ('outer',) | ('st', face, shift)
        | ('zero',), as interpolateValuesAround would decide (hpp:156-198)."""
        g = self.grid
        direction = (self.basis[0][s], self.basis[1][s], self.basis[2][s])
        plan = []
        for it in range(len(g.P)):
            row, outer = [], []
            for k in range(6):
                dx = -self.tau * self.L[s][k]
                shift = _mul(direction, dx)
                t = g.find_cell(it, shift)
                if len(t) == 4:
                    row.append(("cell", t, _add(g.P[it], shift)))
                elif len(t) == 0 or (len(t) in (2, 3) and not g.inner[it]):
                    row.append(("outer",))
                    outer.append(k)
                elif len(t) == 3:
                    row.append(("st", t, shift))
                elif len(t) == 2:
                    raise ValueError("This did not occur ever before")
                else:
                    row.append(("zero",))
            if g.inner[it]:
                if outer:
                    raise ValueError("outer invariant at an inner node")
            elif outer != RIGHT and outer != LEFT and len(outer) != 6 and outer:
                if set(outer) & set(RIGHT):
                    outer = sorted(set(outer) | set(RIGHT))
                if set(outer) & set(LEFT):
                    outer = sorted(set(outer) | set(LEFT))
                for k in outer:
                    row[k] = ("outer",)
            if not g.inner[it]:
                self.outers[s][it] = list(outer)
            plan.append(row)
        return plan

    def _interp(self, it, k, foot, w, wn, grads):
        g = self.grid
        kind = foot[0]
        if kind == "cell":
            verts, q = foot[1], foot[2]
            c = [g.P[x] for x in verts]
            v = [w[x][k] for x in verts]
            gr = [(grads[x][0][k], grads[x][1][k], grads[x][2][k]) for x in verts]
            return tet_hybrid(c, v, gr, q)  # TetrahedronInterpolator::hybridInterpolate
        if kind == "st":  # common.hpp:102-129
            face, shift = foot[1], foot[2]
            r0 = g.P[it]
            r1, r2, r3 = (g.P[x] for x in face)
            rc = _line_flat(r1, r2, r3, r0, _add(r0, shift))
            ww = _lls32(_sub(r2, r1), _sub(r3, r1), _sub(rc, r1))
            pts = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 1)]
            vals = [w[face[0]][k], w[face[1]][k], w[face[2]][k],
                    wn[face[0]][k], wn[face[1]][k], wn[face[2]][k]]
            qst = (ww[0], ww[1], 1 - _length(_sub(rc, r0)) / _length(shift))
            return tet_interpolate_in_owner(pts, vals, qst)  # TetrahedronInterpolator::interpolateInOwner
        return 0.0

    def _mat_vec(self, M, x):  # linal/operators.hpp:109-123
        out = []
        for c in range(9):
            s = M[c][0] * x[0]
            for j in range(1, 9):
                s += M[c][j] * x[j]
            out.append(s)
        return out

    def stage_nodes(self, s):
        """beforeStage + contactAndBorderStage (engine/simplex/Engine.cpp:119-127)."""
        g = self.grid
        n = len(g.P)
        self._w = w = [self._mat_vec(self.U[s], self.u[i]) for i in range(n)]
        self._grads = g.gradients(w)
        self.wn = [[0.0] * 9 for _ in range(n)]
        for it in g.contact_idx + g.border_idx:
            self._node(s, it)

    def stage_finish(self, s, t_next=None):
        """border correctors, innerStage, afterStage + swap (Engine.cpp:128-143)."""
        g = self.grid
        if self.corrected:
            self._correct(s, self.wn, self.time + self.tau if t_next is None else t_next)
        for it in g.inner_idx:
            self._node(s, it)
        self.u = [self._mat_vec(self.U1[s], self.wn[i]) for i in range(len(g.P))]

    def _node(self, s, it):
        for k in range(9):
            if k >= 6:
                self.wn[it][k] = self._w[it][k]
            else:
                self.wn[it][k] = self._interp(it, k, self.feet[s][it][k], self._w, self.wn,
                                              self._grads)

    def stage(self, s, t_next=None):
        """gcmStage with PRODUCT splitting (engine/simplex/Engine.cpp:119-135)."""
        self.stage_nodes(s)
        self.stage_finish(s, t_next)

    def step(self):
        """simplex::Engine::nextTimeStep (Engine.cpp:95-116) + the Clock tick."""
        t_next = self.time + self.tau
        self._plain_correction(t_next)
        for s in range(3):
            self.stage(s, t_next)
        self.time = self.time + self.tau


# ------------------------------------------------------- contact correctors --
# engine/simplex/ContactCorrector.hpp (ContactCorrectorInRiemannInvariants over
# ContactCorrectorInPdeVectors, AdhesionContactMatrixCreator), the two-body
# calculateOuterWaveCorrection (common.hpp:220-260), ElasticModel's global-basis
# border matrices and plain contact corrections (ElasticModel.hpp:157-300), and
# the 6 x 6 determinant / solve of util/math/GslUtils.hpp through GSL's LU
# (gsl_linalg_LU_decomp / _det / _solve; GSL is absent and not vendored: the
# classic Doolittle algorithm with partial pivoting is restated -- unpinned).

def _b1_global():  # borderMatrixFixedVelocityGlobalBasis (ElasticModel.hpp:183-194)
    return [[1.0 if k == i else 0.0 for k in range(9)] for i in range(3)]


def _b2_global(n):  # borderMatrixFixedForceGlobalBasis (ElasticModel.hpp:162-176)
    B = []
    for i in range(3):
        row = [0.0] * 9
        for j in range(3):
            row[_sym(i, j)] = n[j]
        B.append(row)
    return B


def _col(v):
    return [[x] for x in v]


def _flat(m):
    return [r[0] for r in m]


def _invert33(m):  # linal/functions.hpp:128-134
    c = [m[1][1] * m[2][2] - m[1][2] * m[2][1], m[0][2] * m[2][1] - m[0][1] * m[2][2],
         m[0][1] * m[1][2] - m[1][1] * m[0][2], m[1][2] * m[2][0] - m[1][0] * m[2][2],
         m[0][0] * m[2][2] - m[0][2] * m[2][0], m[0][2] * m[1][0] - m[0][0] * m[1][2],
         m[1][0] * m[2][1] - m[1][1] * m[2][0], m[0][1] * m[2][0] - m[0][0] * m[2][1],
         m[0][0] * m[1][1] - m[0][1] * m[1][0]]
    det = _det33(m)
    return [[c[3 * i + j] / det for j in range(3)] for i in range(3)]


def contact_wave_correction(uA, OmegaA, B1A, B2A, uB, OmegaB, B1B, B2B, min1, min2):
    """(det1, det2, successful, valueA, valueB) -- common.hpp:220-260."""
    zero = [0.0] * 9
    R1 = _mat_mul(B1A, OmegaA)
    det1 = abs(_det33(R1))
    if not det1 > min1:
        return det1, 0.0, False, zero, zero
    R = _invert33(R1)
    b1B, b1A = _flat(_mat_mul(B1B, _col(uB))), _flat(_mat_mul(B1A, _col(uA)))
    p = _flat(_mat_mul(R, _col([b1B[i] - b1A[i] for i in range(3)])))
    Q = _mat_mul(R, _mat_mul(B1B, OmegaB))
    B2OB, B2OA = _mat_mul(B2B, OmegaB), _mat_mul(B2A, OmegaA)
    B2OAQ = _mat_mul(B2OA, Q)
    A = [[B2OB[i][j] - B2OAQ[i][j] for j in range(3)] for i in range(3)]
    t = _flat(_mat_mul(B2OA, _col(p)))
    b2A, b2B = _flat(_mat_mul(B2A, _col(uA))), _flat(_mat_mul(B2B, _col(uB)))
    f = [(t[i] + b2A[i]) - b2B[i] for i in range(3)]
    det2 = abs(_det33(A))
    if not det2 > min2:
        return det1, det2, False, zero, zero
    alphaB = list(_solve3(A, f))
    Qa = _flat(_mat_mul(Q, _col(alphaB)))
    alphaA = [p[i] + Qa[i] for i in range(3)]
    return (det1, det2, True, _flat(_mat_mul(OmegaA, _col(alphaA))),
            _flat(_mat_mul(OmegaB, _col(alphaB))))


def _gsl_lu_decomp(A):
    """gsl_linalg_LU_decomp: returns (LU, permutation, signum)."""
    N = len(A)
    A = [list(r) for r in A]
    perm = list(range(N))
    signum = 1
    for j in range(N - 1):
        mx, piv = abs(A[j][j]), j
        for i in range(j + 1, N):
            if abs(A[i][j]) > mx:
                mx, piv = abs(A[i][j]), i
        if piv != j:
            A[j], A[piv] = A[piv], A[j]
            perm[j], perm[piv] = perm[piv], perm[j]
            signum = -signum
        ajj = A[j][j]
        if ajj != 0.0:
            for i in range(j + 1, N):
                aij = A[i][j] / ajj
                A[i][j] = aij
                for k in range(j + 1, N):
                    A[i][k] = A[i][k] - aij * A[j][k]
    return A, perm, signum


def _gsl_lu_det(LU, signum):
    det = float(signum)
    for i in range(len(LU)):
        det *= LU[i][i]
    return det


def _gsl_lu_solve(LU, perm, b):
    N = len(LU)
    x = [b[perm[i]] for i in range(N)]          # gsl_permute_vector
    for i in range(1, N):                       # dtrsv lower, unit
        t = x[i]
        for j in range(i):
            t -= LU[i][j] * x[j]
        x[i] = t
    x[N - 1] = x[N - 1] / LU[N - 1][N - 1]      # dtrsv upper, non-unit
    for i in range(N - 2, -1, -1):
        t = x[i]
        for j in range(i + 1, N):
            t -= LU[i][j] * x[j]
        x[i] = t / LU[i][i]
    return x


def outer_wave_correction_gsl(u, Omega, B, b, min_valid):
    """The one-body calculateOuterWaveCorrection (common.hpp:179-197) for N > 3."""
    M = _mat_mul(B, Omega)
    LU, perm, sg = _gsl_lu_decomp(M)
    det = abs(_gsl_lu_det(LU, sg))
    if not det > min_valid:
        return det, False, [0.0] * 9
    Bu = _flat(_mat_mul(B, _col(u)))
    alpha = _gsl_lu_solve(LU, perm, [b[i] - Bu[i] for i in range(len(b))])
    return det, True, _flat(_mat_mul(Omega, _col(alpha)))


def _sigma_local(u, S):
    sg = [[u[_sym(i, j)] for j in range(3)] for i in range(3)]
    ST = [[S[j][i] for j in range(3)] for i in range(3)]
    return _mat_mul(_mat_mul(ST, sg), S)


def _sigma_global(u, S, sl):
    ST = [[S[j][i] for j in range(3)] for i in range(3)]
    sg = _mat_mul(_mat_mul(S, sl), ST)
    for i in range(3):
        for j in range(3):
            u[_sym(i, j)] = sg[i][j]


def plain_contact_average(uA, uB, normal):  # ElasticModel.hpp:239-272
    uA, uB = list(uA), list(uB)
    v = [(uA[i] + uB[i]) / 2 for i in range(3)]
    uA[:3], uB[:3] = v, list(v)
    S = local_basis(normal)
    lA, lB = _sigma_local(uA, S), _sigma_local(uB, S)
    sn = [(lA[i][2] + lB[i][2]) / 2 for i in range(3)]
    for l in (lA, lB):
        for i in range(3):
            l[i][2] = sn[i]
        for j in range(3):
            l[2][j] = sn[j]
    _sigma_global(uA, S, lA)
    _sigma_global(uB, S, lB)
    return uA, uB


def plain_contact_one_sided(uA, uB, normal):  # ElasticModel.hpp:279-300
    uA = list(uA)
    uA[:3] = uB[:3]
    S = local_basis(normal)
    lA, lB = _sigma_local(uA, S), _sigma_local(uB, S)
    sn = [lB[i][2] for i in range(3)]
    for i in range(3):
        lA[i][2] = sn[i]
    for j in range(3):
        lA[2][j] = sn[j]
    _sigma_global(uA, S, lA)
    return uA


class MultiEngine:
    """simplex::Engine<3> with several bodies of one triangulation and ADHESION
    contacts between them (engine/simplex/Engine.cpp:14-48, 95-287).

    bodies: list (ascending ids) of dicts {"id", "coords", "cells", "global" (local ->
    triangulation vertex), "U", "U1", "L", "pde"} -- the mesh is input data."""

    def __init__(self, bodies, basis, courant, border_conditions=()):
        faces = {}
        for b in bodies:
            for c in b["cells"]:
                for i in range(4):
                    f = tuple(sorted(int(b["global"][c[(i + k) % 4]]) for k in (1, 2, 3)))
                    faces.setdefault(f, []).append(int(b["id"]))
        empty_vertices = set()
        face_grids = []
        for b in bodies:
            glob = [int(x) for x in b["global"]]
            g0 = Grid(b["coords"], b["cells"])  # topology only
            fg = {}
            for ci, c in enumerate(g0.cells):
                for i in range(4):
                    if g0.nb[ci][i] < 0:
                        f = tuple(sorted(glob[c[(i + k) % 4]] for k in (1, 2, 3)))
                        others = [x for x in faces[f] if x != int(b["id"])]
                        fg[(ci, i)] = others[0] if others else EMPTY
                        if not others:
                            empty_vertices.update(f)
            face_grids.append(fg)
        owners = {}
        for b in bodies:
            for g in b["global"]:
                owners.setdefault(int(g), set()).add(int(b["id"]))
        self.bodies = []
        grids = []
        for b, fg in zip(bodies, face_grids):
            glob = [int(x) for x in b["global"]]
            other = []
            for g in glob:
                o = sorted(owners[g] - {int(b["id"])})
                if g in empty_vertices:
                    o = [EMPTY] + o
                other.append(o)
            grids.append(Grid(b["coords"], b["cells"], lambda ci, i, fg=fg: fg[(ci, i)], other))
        tau = None
        for b, g in zip(bodies, grids):   # Engine::estimateTimeStep: minimal over bodies
            mx = max(abs(float(x)) for s in range(3) for x in b["L"][s])
            t = courant * g.average_height / mx
            tau = t if tau is None or t < tau else tau
        self.tau = tau
        for b, g in zip(bodies, grids):
            self.bodies.append(Engine(b["coords"], b["cells"], b["U"], b["U1"], b["L"], basis,
                                      courant, b["pde"], border_conditions, grid=g, tau=tau))
        self.ids = [int(b["id"]) for b in bodies]
        self.globals = [[int(x) for x in b["global"]] for b in bodies]
        self.basis = [[float(basis[r][c]) for c in range(3)] for r in range(3)]
        self.contacts = []
        for ia in range(len(bodies)):       # Utils::makePairs + addContactNode
            for ib in range(ia + 1, len(bodies)):
                self.contacts.append(self._contact(ia, ib))
        self.time = 0.0
        for c in self.contacts:             # applyPlainBorderContactCorrection(0)
            self._plain(c)
        # (each body's Engine already applied its border plain correction at t = 0)

    def _contact(self, ia, ib):
        A, B = self.bodies[ia], self.bodies[ib]
        la = {g: i for i, g in enumerate(self.globals[ia])}
        lb = {g: i for i, g in enumerate(self.globals[ib])}
        pairs = []
        for g in sorted(set(la) & set(lb)):
            a, b = la[g], lb[g]
            if A.grid.other_grids[a] != [self.ids[ib]]:
                continue
            n = A.grid.contact_normal(a, self.ids[ib])
            if n != (0.0, 0.0, 0.0):
                pairs.append((a, b, n))
        min_det = {}
        if pairs:                            # getMaximalPossibleDeterminants (hpp:250-276)
            for s in range(3):
                d = (self.basis[0][s], self.basis[1][s], self.basis[2][s])
                B1, B2 = _b1_global(), _b2_global(d)
                d1, d2, ok, _, _ = contact_wave_correction(
                    [0.0] * 9, A._omega(s, LEFT), B1, B2, [0.0] * 9, B._omega(s, RIGHT), B1, B2, 0, 0)
                if not (ok and d1 > 0 and d2 > 0):
                    raise ValueError("degenerate contact system")
                min_det[s] = (1e-3 * d1, 1e-3 * d2)
        return {"a": ia, "b": ib, "pairs": pairs, "min_det": min_det}

    def _plain(self, c):
        A, B = self.bodies[c["a"]], self.bodies[c["b"]]
        for a, b, n in c["pairs"]:
            A.u[a], B.u[b] = plain_contact_average(A.u[a], B.u[b], n)

    def _correct(self, c, s):
        """ContactCorrectorInRiemannInvariants::applyInGlobalBasis (hpp:333-348)."""
        A, B = self.bodies[c["a"]], self.bodies[c["b"]]
        min1, min2 = c["min_det"].get(s, (0.0, 0.0))
        both = sorted(LEFT + RIGHT)
        for a, b, n in c["pairs"]:
            oa, ob = list(A.outers[s].get(a, [])), list(B.outers[s].get(b, []))
            N = (len(oa) + len(ob)) // 3    # matchInnersAndOuters (hpp:365-397)
            if N % 2 == 1:
                if N == 3:
                    oa, ob = list(both), list(both)
                elif not oa:
                    oa = RIGHT if ob == LEFT else LEFT
                else:
                    ob = RIGHT if oa == LEFT else LEFT
                for i in oa:
                    A.wn[a][i] = 0
                for i in ob:
                    B.wn[b][i] = 0
            uA = A._mat_vec(A.U1[s], A.wn[a])
            uB = B._mat_vec(B.U1[s], B.wn[b])
            B1, B2 = _b1_global(), _b2_global(n)
            if len(oa) == 3 and len(ob) == 3:
                _, _, ok, vA, vB = contact_wave_correction(uA, A._omega(s, oa), B1, B2,
                                                           uB, B._omega(s, ob), B1, B2, min1, min2)
                if ok:
                    uA = [uA[i] + vA[i] for i in range(9)]
                    uB = [uB[i] + vB[i] for i in range(9)]
                else:
                    uA, uB = plain_contact_average(uA, uB, n)
            elif (len(oa) == 6 and not ob) or (len(ob) == 6 and not oa):
                X, uX, uY = (A, uA, uB) if oa else (B, uB, uA)
                Bm = B1 + B2
                b12 = _flat(_mat_mul(B1, _col(uY))) + _flat(_mat_mul(B2, _col(uY)))
                Om = [X._omega(s, RIGHT)[i] + X._omega(s, LEFT)[i] for i in range(9)]
                _, ok, v = outer_wave_correction_gsl(uX, Om, Bm, b12, min1)
                uX = [uX[i] + v[i] for i in range(9)] if ok else plain_contact_one_sided(uX, uY, n)
                if oa:
                    uA = uX
                else:
                    uB = uX
            else:
                r1 = contact_wave_correction(uA, A._omega(s, RIGHT), B1, B2,
                                             uB, B._omega(s, LEFT), B1, B2, min1, min2)
                r2 = contact_wave_correction(uA, A._omega(s, LEFT), B1, B2,
                                             uB, B._omega(s, RIGHT), B1, B2, min1, min2)
                if r1[2] and r2[2]:
                    uA = [uA[i] + (r1[3][i] + r2[3][i]) / 2 for i in range(9)]
                    uB = [uB[i] + (r1[4][i] + r2[4][i]) / 2 for i in range(9)]
                else:
                    uA, uB = plain_contact_average(uA, uB, n)
            A.wn[a] = A._mat_vec(A.U[s], uA)
            B.wn[b] = B._mat_vec(B.U[s], uB)

    def step(self):
        """simplex::Engine::nextTimeStep (Engine.cpp:95-116)."""
        t_next = self.time + self.tau
        for c in self.contacts:
            self._plain(c)
        for e in self.bodies:
            e._plain_correction(t_next)
        for s in range(3):
            for e in self.bodies:
                e.stage_nodes(s)
            for c in self.contacts:
                self._correct(c, s)
            for e in self.bodies:
                e.stage_finish(s, t_next)
        self.time = self.time + self.tau
        for e in self.bodies:
            e.time = self.time
