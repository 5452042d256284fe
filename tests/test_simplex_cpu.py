"""Simplex path without a GPU: the product's host set-up (gcm_amd._gcm_host.simplex_plans:
mesh, time step, feet of every characteristic, outer invariants) against the
oracle's independent restatement of SimplexGrid's line walk and
GridCharacteristicMethodInRiemannInvariants::interpolateValuesAround, plus the
mesh invariants the reference's own grid test checks (TestSimplexGrid.cpp:51-91:
inner nodes have a zero border normal, border normals of a cube point along the
face normals within 0.3).  Reference numerics parity is unpinned (CGAL absent)."""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle import simplex as S
from tests.simplex_spec import host_task, oracle_engine

KIND = {"cell": 0, "outer": 1, "st": 2, "zero": 3}


@pytest.fixture(scope="module")
def H():
    from gcm_amd import _gcm_host
    return _gcm_host


@pytest.mark.parametrize("n,courant,jitter,seed", [(3, 1.0, 0.0, 0), (4, 1.0, 0.1, 7),
                                                   (4, 2.0, 0.1, 7), (5, 1.7, 0.15, 3)])
def test_plans_match_oracle(H, n, courant, jitter, seed):
    p = H.simplex_plans(host_task(n, courant, jitter, seed))
    e = oracle_engine(p, courant)
    assert e.tau == p["tau"]
    assert e.grid.border_idx == list(p["border"]) and e.grid.inner_idx == list(p["inner"])
    U, U1, _ = O.isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
    assert np.array_equal(U, p["U"]) and np.array_equal(U1, p["U1"])
    for s in range(3):
        st = p["stages"][s]
        for it in range(len(p["coords"])):
            for k in range(6):
                f = e.feet[s][it][k]
                assert int(st["kind"][it, k]) == KIND[f[0]], (s, it, k)
                if f[0] == "cell":
                    assert list(st["v"][it, k]) == list(f[1])
                    lam = S.barycentric4(*[e.grid.P[x] for x in f[1]], f[2])
                    assert np.array_equal(np.array(lam), st["lam"][it, k])
                    assert np.array_equal(np.array(f[2]), st["q"][it, k])
                elif f[0] == "st":
                    assert list(st["v"][it, k][:3]) == list(f[1])


def test_mesh_invariants(H):
    p = H.simplex_plans(host_task(5, 1.0, 0.12, 11))
    P, C = p["coords"], p["cells"]
    for c in C:
        assert S.oriented_volume(*[tuple(P[x]) for x in c]) > 0
    assert len(p["border"]) + len(p["inner"]) == len(P) == 6 ** 3
    assert len(p["inner"]) == 4 ** 3
    # the box's faces stay planar: border nodes lie on the unit cube's faces
    for it in p["border"]:
        x = P[it]
        assert any(x[i] == 0.0 or x[i] == 1.0 for i in range(3))


def test_zero_crossing_invariants_are_exact_hits(H):
    """Invariants 6..8 have L = 0: no foot is resolved for them (hpp:166-170)."""
    p = H.simplex_plans(host_task(3))
    assert p["stages"][0]["kind"].shape[1] == 6


def test_uncompilable_configurations_are_refused(H):
    t = host_task(3)
    t.calculation_basis = []
    with pytest.raises(Exception):
        H.simplex_plans(t)  # random basis per step: not on this path


def test_oracle_zero_state_stays_zero(H):
    """TestSimplexGcm.cpp:29-53 (ZeroInitialization) on the oracle."""
    p = H.simplex_plans(host_task(3, pressure=0.0))
    e = oracle_engine(p, 1.0)
    for _ in range(3):
        e.step()
    assert all(v == 0.0 for row in e.u for v in row)


def test_oracle_uniform_field_is_preserved_inside():
    """A homogeneous state is a solution: every inner-node invariant
    interpolates a constant exactly up to rounding (sanity of the restatement)."""
    from gcm_amd import _gcm_host as H
    vec = [0.3, -0.2, 0.1, 1.0, 0.5, -0.25, 2.0, 0.75, -1.5]
    p = H.simplex_plans(host_task(4, 0.8, 0.1, 5, pressure=0.0, vector=vec))
    e = oracle_engine(p, 0.8)
    e.stage(0)
    for it in e.grid.inner_idx:
        for k in range(9):
            assert math.isclose(e.u[it][k], p["pde"][it][k], rel_tol=1e-12, abs_tol=1e-12)


# ------------------------------------------------------------ border correctors --

from tests.simplex_spec import FREE_BORDER, MIXED_BORDER  # noqa: E402

CODE = {(1, 3, 5): 1, (0, 2, 4): 2}


@pytest.mark.parametrize("border", [FREE_BORDER, MIXED_BORDER], ids=["free", "mixed"])
@pytest.mark.parametrize("n,courant,jitter,seed", [(4, 1.0, 0.1, 7), (5, 1.7, 0.15, 3)])
def test_border_plan_matches_oracle(H, border, n, courant, jitter, seed):
    """Engine::addBorderNode's choice of nodes / conditions / normals, the border
    matrices, local bases, thresholds and wave indices: host == oracle exactly."""
    p = H.simplex_plans(host_task(n, courant, jitter, seed, border=border))
    e = oracle_engine(p, courant, border)
    b = p["border_plan"]
    assert list(b["nodes"]) == [x[0] for x in e.corrected]
    assert list(b["cond"]) == [x[1] for x in e.corrected]
    kinds = [c[1] for c in border]
    assert list(b["type"]) == [0 if k == "FIXED_FORCE" else 1 for k in kinds]
    nn = len(e.corrected)
    for i, (it, ci, nrm) in enumerate(e.corrected):
        assert tuple(b["normal"][3 * i:3 * i + 3]) == nrm
        B = S.border_matrix(kinds[ci], nrm)
        assert list(b["B"][27 * i:27 * i + 27]) == [x for row in B for x in row]
        Sb = S.local_basis(nrm)
        assert list(b["S"][9 * i:9 * i + 9]) == [x for row in Sb for x in row]
        for s in range(3):
            outers = tuple(e.outers[s].get(it, []))
            want = CODE.get(outers, 0 if not outers else 3)
            assert b["outer"][s * nn + i] == want
    for (ci, s), v in e.min_det.items():
        assert b["min_det"][3 * ci + s] == v
    if border is MIXED_BORDER:
        assert 0 < sum(b["cond"]) < nn   # both conditions own nodes


def test_outer_wave_correction_satisfies_the_condition():
    """calculateOuterWaveCorrection's purpose (common.hpp:170-185): after adding
    Omega * alpha the border condition B u = b holds (to rounding)."""
    U, U1, _ = O.isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
    rng = np.random.default_rng(5)
    for kind in ("FIXED_FORCE", "FIXED_VELOCITY"):
        for _ in range(20):
            nrm = S._normalize(tuple(rng.normal(size=3)))
            u = list(rng.uniform(-1, 1, 9))
            b = list(rng.uniform(-1, 1, 3))
            B = S.border_matrix(kind, nrm)
            omega = [[U1[0][i][c] for c in S.RIGHT] for i in range(9)]
            det, ok, v = S.outer_wave_correction(u, omega, B, b, 0.0)
            assert ok and det > 0
            uc = [u[i] + v[i] for i in range(9)]
            Bu = [sum(B[r][k] * uc[k] for k in range(9)) for r in range(3)]
            assert np.allclose(Bu, b, atol=1e-12)


def test_plain_correction_sets_local_traction_and_velocity():
    """applyPlainBorderCorrection (ElasticModel.hpp:202-228): sigma in the local
    basis has the given last row / column; velocity = S * value."""
    rng = np.random.default_rng(9)
    nrm = S._normalize(tuple(rng.normal(size=3)))
    Sb = np.array(S.local_basis(nrm))
    u = list(rng.uniform(-1, 1, 9))
    val = [0.3, -0.2, 0.7]
    uf = S.plain_border_correction(u, "FIXED_FORCE", nrm, val)
    sig = np.array([[uf[S._sym(i, j)] for j in range(3)] for i in range(3)])
    loc = Sb.T @ sig @ Sb
    assert np.allclose(loc[:, 2], val, atol=1e-12) and np.allclose(loc[2, :], val, atol=1e-12)
    assert uf[:3] == u[:3]
    uv = S.plain_border_correction(u, "FIXED_VELOCITY", nrm, val)
    assert np.allclose(uv[:3], Sb @ np.array(val), atol=1e-15) and uv[3:] == u[3:]


def test_border_condition_validation(H):
    t = host_task(3, border=[(("infinite",), "FIXED_FORCE", (lambda t: 0.0,) * 2, True)])
    with pytest.raises(Exception, match="OUTER_NUMBER"):
        H.simplex_plans(t)
    with pytest.raises(Exception, match="unknown border condition type"):
        host_task(3, border=[(("infinite",), "FIXED_STRAIN", (lambda t: 0.0,) * 3, True)])


# ---- BASELINE config 5: the layer with a fracture (cavity) ---------------------

from tests.simplex_spec import FRACTURE_OFF, FREE_BORDER, fracture_task  # noqa: E402


def _read_off(path):
    toks = []
    for line in open(path):
        toks += line.split("#")[0].split()
    assert toks[0] == "OFF"
    nv, nf = int(toks[1]), int(toks[2])
    pts = np.array(toks[4:4 + 3 * nv], dtype=float).reshape(nv, 3)
    f = np.array(toks[4 + 3 * nv:], dtype=int).reshape(nf, 4)
    assert (f[:, 0] == 3).all()
    return pts, f[:, 1:]


def _inside_by_ray(pts, faces, q, d=(0.5773, 0.5781, 0.5761)):
    """Crossing parity of a ray (Moller-Trumbore): an independent inside test."""
    d = np.array(d)
    n = 0
    for a, b, c in faces:
        A, B, C = pts[a], pts[b], pts[c]
        e1, e2 = B - A, C - A
        h = np.cross(d, e2)
        det = e1 @ h
        if abs(det) < 1e-15:
            continue
        s = q - A
        u = (s @ h) / det
        qq = np.cross(s, e1)
        v = (d @ qq) / det
        t = (e2 @ qq) / det
        if u >= 0 and v >= 0 and u + v <= 1 and t > 0:
            n += 1
    return n % 2 == 1


def test_fracture_off_fixture():
    """meshes/layers_with_fracture.off: the 12 + 4 triangles of the layer box and the
    fracture tetrahedron (12 vertices)."""
    pts, faces = _read_off(FRACTURE_OFF)
    assert pts.shape == (12, 3) and faces.shape == (16, 3)
    assert pts[:8].min(0).tolist() == [0, 0, 0] and pts[:8].max(0).tolist() == [0.16, 0.16, 0.04]


def test_fracture_mesh_is_carved(H):
    """Cells whose centroid lies in the fracture are empty space: the kept cells'
    centroids are inside the domain, every box cell missing from the mesh is in the
    fracture, and the nodes around the cavity are border nodes."""
    n = (16, 16, 8)
    p = H.simplex_plans(fracture_task(n))
    pts, faces = _read_off(FRACTURE_OFF)
    P, C = p["coords"], p["cells"]
    cen = P[C].mean(axis=1)
    assert len(C) < 6 * n[0] * n[1] * n[2]
    for q in cen[::97]:
        assert _inside_by_ray(pts, faces, q)
    # the border nodes that are not on the box surface surround the fracture
    box = np.array([0.16, 0.16, 0.04])
    inner_border = [i for i in p["border"] if np.all(P[i] > 0) and np.all(P[i] < box)]
    assert len(inner_border) > 0
    lo, hi = pts[8:].min(0) - 0.02, pts[8:].max(0) + 0.02
    for i in inner_border:
        assert np.all(P[i] >= lo) and np.all(P[i] <= hi)
    # every vertex of the triangulation that survives keeps its cells
    assert len(p["border"]) + len(p["inner"]) == len(P)


@pytest.mark.parametrize("courant", [1.0, 1.7])
def test_fracture_plans_match_oracle(H, courant):
    p = H.simplex_plans(fracture_task((16, 16, 8), courant))
    e = oracle_engine(p, courant, FREE_BORDER)
    assert e.tau == p["tau"]
    assert e.grid.border_idx == list(p["border"]) and e.grid.inner_idx == list(p["inner"])
    for s in range(3):
        st = p["stages"][s]
        for it in range(len(p["coords"])):
            for k in range(6):
                f = e.feet[s][it][k]
                assert int(st["kind"][it, k]) == KIND[f[0]], (s, it, k)
                if f[0] == "cell":
                    assert list(st["v"][it, k]) == list(f[1])
    assert len(e.corrected) == len(p["border_plan"]["nodes"])


# ---- two bodies, ADHESION contact correctors ---------------------------------

from tests.simplex_spec import LAYER_MATERIALS, layered_task, oracle_multi  # noqa: E402


@pytest.mark.parametrize("n,courant", [(5, 1.0), (6, 1.7)])
def test_layered_contact_plans_match_oracle(H, n, courant):
    """Body meshes, node states, time step, contact node pairs and normals, and the
    per-stage wave codes after matchInnersAndOuters: product == oracle."""
    p = H.simplex_plans(layered_task(n, courant))
    o = oracle_multi(p, courant)
    assert o.tau == p["tau"]
    assert len(p["bodies"]) == 2 and len(p["contacts"]) == 1
    for b, e in zip(p["bodies"], o.bodies):
        g = e.grid
        assert g.inner_idx == list(b["inner"]) and g.border_idx == list(b["border"])
        assert g.contact_idx == list(b["contact"]) and len(b["contact"]) > 0
        assert [x[0] for x in e.corrected] == list(b["border_plan"]["nodes"])
        assert np.array_equal(np.array([x[2] for x in e.corrected]).ravel(),
                              np.array(b["border_plan"]["normal"]))
        U, U1, _ = O.isotropic_elastic_matrices(3, *LAYER_MATERIALS[int(b["id"])])
        assert np.array_equal(U1, b["U1"])
    c, oc = p["contacts"][0], o.contacts[0]
    assert list(c["nodes_a"]) == [x[0] for x in oc["pairs"]]
    assert list(c["nodes_b"]) == [x[1] for x in oc["pairs"]]
    assert np.array_equal(np.array(c["normal"]), np.array([x[2] for x in oc["pairs"]]).ravel())
    assert c["min_det"] == [oc["min_det"][s][k] for s in range(3) for k in range(2)]
    nn = len(c["nodes_a"])
    code = {(): 0, (1, 3, 5): 1, (0, 2, 4): 2, (0, 1, 2, 3, 4, 5): 3}
    size = {0: 0, 1: 3, 2: 3, 3: 6}

    def match(ca, cb):  # matchInnersAndOuters (ContactCorrector.hpp:365-397)
        N = (size[ca] + size[cb]) // 3
        if N % 2 == 0:
            return ca, cb
        if N == 3:
            return 3 | 4, 3 | 4
        if ca == 0:
            return (1 if cb == 2 else 2) | 4, cb | 4
        return ca | 4, (1 if ca == 2 else 2) | 4

    A, B = o.bodies
    for s in range(3):
        for i, (a, b, _) in enumerate(oc["pairs"]):
            want = match(code[tuple(A.outers[s].get(a, []))], code[tuple(B.outers[s].get(b, []))])
            assert (c["code_a"][s * nn + i], c["code_b"][s * nn + i]) == want
    # branch coverage of the configuration: the 3+3 system and the 6 x 6 (GSL) one
    codes = {(c["code_a"][k] & 3, c["code_b"][k] & 3) for k in range(3 * nn)}
    assert any(x in codes for x in [(1, 2), (2, 1)])
    assert any(x in codes for x in [(3, 0), (0, 3)])


def test_gsl_lu_restatement():
    """The oracle's GSL LU (determinant, solve) against numpy on random 6 x 6 systems."""
    rng = np.random.default_rng(3)
    for _ in range(20):
        A = rng.standard_normal((6, 6))
        b = rng.standard_normal(6)
        LU, perm, sg = S._gsl_lu_decomp(A.tolist())
        assert abs(S._gsl_lu_det(LU, sg) - np.linalg.det(A)) < 1e-9 * abs(np.linalg.det(A)) + 1e-12
        x = S._gsl_lu_solve(LU, perm, b.tolist())
        assert np.allclose(A @ np.array(x), b, atol=1e-9)


def test_plain_contact_average_satisfies_adhesion():
    """applyPlainContactCorrectionAsAverage: equal velocities and equal normal
    tractions afterwards."""
    rng = np.random.default_rng(5)
    n = np.array([0.3, -0.4, 0.866])
    n = n / np.linalg.norm(n)
    uA, uB = S.plain_contact_average(rng.standard_normal(9).tolist(), rng.standard_normal(9).tolist(),
                                     tuple(n))
    sig = lambda u: np.array([[u[3], u[4], u[5]], [u[4], u[6], u[7]], [u[5], u[7], u[8]]])
    assert np.allclose(uA[:3], uB[:3])
    assert np.allclose(sig(uA) @ n, sig(uB) @ n)


def test_simplex_vtu_snapshot(H, tmp_path):
    """VtkSnapshotter of a simplex body (VtkSnapshotter.hpp:20-61, VtkUtils.hpp:54-66,
    140-160): an UnstructuredGrid of VTK_TETRA cells over the mesh vertices with
    "Velocity", the quantities to snap and "material_index" (Float32)."""
    from tests.helpers import read_vtu
    t = layered_task(4, 1.0)
    t.set_vtk_quantities(["PRESSURE", "Sxy"])
    p = H.simplex_plans(t)
    for body in (0, 1):
        b = p["bodies"][body]
        path = str(tmp_path / f"s{body}.vtu")
        rng = np.random.default_rng(body)
        layer = rng.standard_normal((len(b["coords"]), 9))
        H.write_simplex_vtk(t, path, layer, body)
        arrays, pts, conn, offs, types = read_vtu(path)
        assert np.array_equal(pts, b["coords"].astype(np.float32))
        assert np.array_equal(conn, b["cells"]) and (types == 10).all()
        assert np.array_equal(offs, 4 * np.arange(1, len(conn) + 1))
        assert list(arrays) == ["Velocity", "pressure", "Sxy", "material_index"]
        assert np.array_equal(arrays["Velocity"], layer[:, :3].astype(np.float32))
        pres = -(layer[:, 3] + layer[:, 6] + layer[:, 8]) / 3
        assert np.array_equal(arrays["pressure"][:, 0], pres.astype(np.float32))
        assert np.array_equal(arrays["Sxy"][:, 0], layer[:, 4].astype(np.float32))


# ---- INM_MESHER ----------------------------------------------------------------

INM_FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "testInmLoader.out")


def test_inm_reader_known_answers(H):
    """TestInmMeshLoader.readFromFile (TestInmMeshLoader.cpp:19-68) on the reference's
    meshes/testInmLoader.out (copied as a fixture)."""
    P, C, M = H.read_inm(INM_FIXTURE)
    assert P.shape == (12, 3) and len(C) == 3
    assert abs(P[3][0] - -2.583210754394531250e+01) < 1e-9
    assert abs(P[4][0] - 2.400143432617187500e+01) < 1e-9
    assert abs(P[11][0] - -6.843022155761718750e+01) < 1e-9
    assert abs(P[0][1] - 4.283624267578125000e+01) < 1e-9
    assert abs(P[11][1] - 3.788503265380859375e+01) < 1e-9
    assert abs(P[0][2] - 1.406894775390625000e+03) < 1e-9
    mats = {tuple(sorted(c)): m for c, m in zip(C, M)}
    assert mats == {(1, 2, 3, 4): 4, (5, 6, 7, 8): 5, (9, 10, 11, 12): 1}


def test_inm_mesher_reproduces_the_triangulation(H, tmp_path):
    """A triangulation written as an INM file and loaded through INM_MESHER gives the
    same bodies, plans and contacts as the mesher that made it."""
    from tests.simplex_spec import write_inm
    t = layered_task(5, 1.3)
    P, C, G = H.simplex_triangulation(t)
    path = tmp_path / "layers.out"
    write_inm(path, P, C, G)
    a, b = H.simplex_plans(t), H.simplex_plans(layered_task(5, 1.3, inm=path))
    assert a["tau"] == b["tau"]
    for x, y in zip(a["bodies"], b["bodies"]):
        for k in ("coords", "cells", "pde", "inner", "border", "contact", "global"):
            assert np.array_equal(np.array(x[k]), np.array(y[k])), k
        for s in range(3):
            assert np.array_equal(x["stages"][s]["kind"], y["stages"][s]["kind"])
            assert np.array_equal(x["stages"][s]["lam"], y["stages"][s]["lam"])
    assert a["contacts"][0]["code_a"] == b["contacts"][0]["code_a"]


def test_inm_mesher_rejects_unknown_materials(H, tmp_path):
    from tests.simplex_spec import write_inm
    P, C, G = H.simplex_triangulation(layered_task(3))
    path = tmp_path / "bad.out"
    write_inm(path, P, C, [7] * len(C))
    with pytest.raises(Exception):
        H.simplex_plans(layered_task(3, inm=path))


# ---- BASELINE config 4: parseTaskCube on meshes/cube.off ----------------------

from tests.simplex_spec import CUBE_BORDER, CUBE_OFF, cube_task  # noqa: E402


def test_cube_off_fixture():
    """meshes/cube.off: the unit cube as 8 vertices and 12 triangles."""
    pts, faces = _read_off(CUBE_OFF)
    assert pts.shape == (8, 3) and faces.shape == (12, 3)
    assert pts.min(0).tolist() == [0, 0, 0] and pts.max(0).tolist() == [1, 1, 1]


def test_cube_task_plans_match_oracle(H):
    """parseTaskCube (main.cpp:547-639) at its spatial step 0.05: the carved mesh
    keeps every cell of the unit cube, the left-face traction condition owns
    exactly the x <= 0.01 border nodes (the last containing condition wins), and
    the border plan (nodes, conditions, normals, matrices, wave codes) equals the
    oracle's decisions."""
    p = H.simplex_plans(cube_task())
    P = p["coords"]
    assert len(P) == 21 ** 3 and len(p["cells"]) == 6 * 20 ** 3
    e = oracle_engine(p, 1.0, CUBE_BORDER)
    assert e.tau == p["tau"]
    b = p["border_plan"]
    assert list(b["nodes"]) == [x[0] for x in e.corrected]
    assert list(b["cond"]) == [x[1] for x in e.corrected]
    left = {int(i) for i, c in zip(b["nodes"], b["cond"]) if c == 1}
    assert left == {int(i) for i in b["nodes"] if P[i][0] <= 0.01}
    assert 0 < len(left) < len(b["nodes"])
    nn = len(e.corrected)
    for s in range(3):
        for i, (it, ci, nrm) in enumerate(e.corrected):
            outers = tuple(e.outers[s].get(it, []))
            assert b["outer"][s * nn + i] == CODE.get(outers, 0 if not outers else 3)


# ---- the reference's own known answers for the simplex numerics -------------
# src/test/sequence/TestInterpolator.cpp:129-282 and TestGslUtils.cpp:76-115,
# restated with fixed seeds (the reference seeds with time(0), Utils.hpp:48-50).
# They pin oracle/simplex.py's interpolators and LU, which the GPU tests compare
# the kernels with bitwise, and the host set-up code that makes the stage plans'
# weights (tet_barycentric, tet_owner_pick) and the contact correctors' LU
# (csrc/contact.hpp through gsl_lu), bitwise against the oracle.

def _rand_pts(rng, n, dim):
    return [tuple(float(x) for x in rng.uniform(-1e6, 1e6, dim)) for _ in range(n)]


def _rand_lam(rng, n):
    lam = rng.uniform(0, 1, n)
    return lam / (lam[0] + lam[1] + lam[2] + (lam[3] if n == 4 else 0.0))


def _f3(x):  # TetrahedronInterpolator.linear's f
    return 5 * x[0] + 8 * x[1] - 4 * x[2] - 2


def _q3(x):  # TetrahedronInterpolator.quadratic's f and its gradient
    return (8 * x[0] * x[0] + 10 * x[0] * x[1] - 9 * x[0] * x[2] - 15 * x[1] * x[1] + 6 * x[1] * x[2]
            - 7 * x[2] * x[2] + 5 * x[0] + 8 * x[1] - 7 * x[2] - 2)


def _g3(x):
    return (16 * x[0] + 10 * x[1] - 9 * x[2] + 5, -30 * x[1] + 10 * x[0] + 6 * x[2] + 8,
            -14 * x[2] + 6 * x[1] - 9 * x[0] - 7)


def _comb(lam, pts):
    d = len(pts[0])
    return tuple(sum(lam[i] * pts[i][k] for i in range(len(pts))) for k in range(d))


def tet_known_answer_cases(n=1000, seed=129):
    """(c, q) pairs as TestInterpolator.cpp:183-264 draws them: four random
    vertices in [-1e6, 1e6]^3 and a random convex combination."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = _rand_pts(rng, 4, 3)
        out.append((c, _comb(_rand_lam(rng, 4), c)))
    return out


def test_tetrahedron_interpolator_linear_known_answers():
    """TetrahedronInterpolator.linear (TestInterpolator.cpp:183-207): exact for a
    linear f within EQUALITY_TOLERANCE * |f(q)|; a point outside throws."""
    for c, q in tet_known_answer_cases():
        v = [_f3(x) for x in c]
        assert abs(S.tet_linear(c, v, q) - _f3(q)) <= S.EQUALITY_TOLERANCE * abs(_f3(q))
        out = tuple(2 * c[0][k] + c[1][k] - c[2][k] - c[3][k] for k in range(3))
        with pytest.raises(ValueError):
            S.tet_linear(c, v, out)


def test_tetrahedron_interpolator_quadratic_known_answers():
    """TetrahedronInterpolator.quadratic (TestInterpolator.cpp:210-244): exact for
    a quadratic f with its gradients; a point outside throws."""
    for c, q in tet_known_answer_cases(seed=210):
        v, g = [_q3(x) for x in c], [_g3(x) for x in c]
        assert abs(S.tet_quadratic(c, v, g, q) - _q3(q)) <= S.EQUALITY_TOLERANCE * abs(_q3(q))
        out = tuple(c[0][k] - c[1][k] - c[2][k] + 2 * c[3][k] for k in range(3))
        with pytest.raises(ValueError):
            S.tet_quadratic(c, v, g, out)


def test_interpolate_in_owner_known_answers(H):
    """TriangleInterpolator / TetrahedronInterpolator.interpolateInOwner
    (TestInterpolator.cpp:178-185, 247-257): the owner holding q has value 1
    at every vertex, the others 1e100 -- the answer is exactly 1.  The host
    pick the stage plans use (tet_owner_pick) == the oracle's, bitwise."""
    assert S.tri_interpolate_in_owner([(0, 0), (0, 1), (1, 0), (1, 1)], [1, 1, 1, 1e100], (0.2, 0.2)) == 1
    c6 = [(0, 0, 0), (0, 1, 0), (1, 0, 0), (0, 0, 1), (0, 1, 1), (1, 0, 1)]
    v6 = [1, 1, 1, 1, 1e100, 1e100]
    assert S.tet_interpolate_in_owner(c6, v6, (0.1, 0.1, 0.1)) == 1
    slots, lam = H.tet_owner_pick([list(map(float, p)) for p in c6], [0.1, 0.1, 0.1])
    tr, lam_o = S.tet_owner_pick(c6, (0.1, 0.1, 0.1))
    assert tuple(slots) == tuple(tr) and tuple(lam) == tuple(lam_o)
    assert lam[0] * v6[slots[0]] + lam[1] * v6[slots[1]] + lam[2] * v6[slots[2]] + lam[3] * v6[slots[3]] == 1
    # the space-time prism of interpolateInSpaceTime (common.hpp:102-129): host == oracle everywhere
    pts = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 1)]
    rng = np.random.default_rng(102)
    for _ in range(300):
        a, b = rng.uniform(0, 1, 2)
        if a + b > 1:
            a, b = 1 - a, 1 - b
        q = (float(a), float(b), float(rng.uniform(0, 1)))
        hs, hl = H.tet_owner_pick([list(map(float, p)) for p in pts], list(q))
        os_, ol = S.tet_owner_pick(pts, q)
        assert tuple(hs) == tuple(os_) and tuple(hl) == tuple(ol)
    with pytest.raises(Exception):
        H.tet_owner_pick([list(map(float, p)) for p in pts], [2.0, 2.0, 0.5])


def test_tetrahedron_barycentric_host_equals_oracle(H):
    """The stage plans' CELL weights (host linal::barycentricCoordinates) ==
    the oracle's, bitwise, on the known-answer cases."""
    for c, q in tet_known_answer_cases(300, seed=142):
        assert tuple(H.tet_barycentric(*[list(x) for x in c], list(q))) == S.barycentric4(*c, q)


def test_quadratic_min_max_known_answers():
    """Triangle / TetrahedronInterpolator.quadraticMinMax (TestInterpolator.cpp:
    267-282): f = |x|^2 with its gradients; the quadratic value at 0 is 0, below
    every vertex value, and the limiter returns exactly 1.  hybridInterpolate
    (what the stage uses) falls back to the linear form there instead: 1.5."""
    assert S.tri_min_max([(0, 1), (1, 0), (-1, -1)], [1, 1, 2], [(0, 2), (2, 0), (-2, -2)], (0, 0)) == 1
    c = [(0, 0, 1), (0, 1, 0), (1, 0, 0), (-1, -1, -1)]
    v, g = [1, 1, 1, 3], [(0, 0, 2), (0, 2, 0), (2, 0, 0), (-2, -2, -2)]
    assert S.tet_min_max(c, v, g, (0, 0, 0)) == 1
    assert S.tet_quadratic(c, v, g, (0, 0, 0)) == 0
    assert S.tet_hybrid(c, v, g, (0, 0, 0)) == 1.5


def test_triangle_interpolator_known_answers():
    """TriangleInterpolator.linear / .quadratic (TestInterpolator.cpp:129-175) on
    the oracle's restatement (the 2-D simplex path is not built: no 2-D config)."""
    rng = np.random.default_rng(129)
    f = lambda x: 5 * x[0] + 8 * x[1] - 2  # noqa: E731
    fq = lambda x: 8 * x[0] * x[0] + 10 * x[0] * x[1] - 15 * x[1] * x[1] + 5 * x[0] + 8 * x[1] - 2  # noqa: E731
    gq = lambda x: (16 * x[0] + 10 * x[1] + 5, -30 * x[1] + 10 * x[0] + 8)  # noqa: E731
    for _ in range(1000):
        c = _rand_pts(rng, 3, 2)
        q = _comb(_rand_lam(rng, 3), c)
        assert abs(S.tri_linear(c, [f(x) for x in c], q) - f(q)) <= S.EQUALITY_TOLERANCE * abs(f(q))
        assert abs(S.tri_quadratic(c, [fq(x) for x in c], [gq(x) for x in c], q) - fq(q)) <= \
            S.EQUALITY_TOLERANCE * abs(fq(q))
        out = tuple(-2 * c[0][k] + c[1][k] + 2 * c[2][k] for k in range(2))
        with pytest.raises(ValueError):
            S.tri_linear(c, [f(x) for x in c], out)
        out = tuple(3 * c[0][k] - c[1][k] - c[2][k] for k in range(2))
        with pytest.raises(ValueError):
            S.tri_quadratic(c, [fq(x) for x in c], [gq(x) for x in c], out)


def test_gsl_utils_known_answers(H):
    """GslUtils.determinant / solveLinearSystem (TestGslUtils.cpp:76-115) through
    the oracle's GSL LU and csrc/contact.hpp's (host instantiation of the code the
    contact kernels run): det(0_5) = 0, det(1_6) = 0, det(I_9) = 1, det(-I_7) =
    -1 exactly; a 9 x 9 Vandermonde determinant within eps = 1e-2 relative
    (GslUtils.hpp:15); 5 I x = 5 * 1 gives x = 1 exactly; a singular 1_5 system is
    refused (gsl_linalg_LU_solve: matrix is singular); random 6 x 6 systems."""
    def odet(A):
        LU, _, sg = S._gsl_lu_decomp(np.asarray(A, dtype=float).tolist())
        return S._gsl_lu_det(LU, sg)
    cases = [(np.zeros((5, 5)), 0.0), (np.ones((6, 6)), 0.0), (np.eye(9), 1.0), (-np.eye(7), -1.0)]
    for A, want in cases:
        assert odet(A) == want
        assert H.gsl_lu(A) == want
    rng = np.random.default_rng(76)
    a = rng.uniform(-1, 1, 9)  # linal::random<Vector<9>>() in [-1, 1]
    V = np.array([[a[i] ** j for j in range(9)] for i in range(9)])
    det = 1.0
    for i in range(9):
        for j in range(i + 1, 9):
            det *= a[j] - a[i]
    assert abs(odet(V) - det) <= abs(det) * 1e-2
    assert H.gsl_lu(V) == odet(V)  # bitwise: the same restated algorithm
    x = H.gsl_lu(5 * np.eye(4), [5.0] * 4)
    assert x == [1.0] * 4
    LU, perm, _ = S._gsl_lu_decomp((5 * np.eye(4)).tolist())
    assert S._gsl_lu_solve(LU, perm, [5.0] * 4) == [1.0] * 4
    with pytest.raises(Exception, match="singular"):
        H.gsl_lu(np.ones((5, 5)), [1.0] * 5)
    for _ in range(200):
        A = rng.uniform(-1e12, 1e12, (6, 6))
        b = rng.uniform(-1e12, 1e12, 6)
        xh = H.gsl_lu(A, b.tolist())
        LU, perm, _ = S._gsl_lu_decomp(A.tolist())
        assert xh == S._gsl_lu_solve(LU, perm, b.tolist())
        # linal::approximatelyEqual(A * x, b): relative 1e-9 per component on the scale of b
        r = A @ np.array(xh) - b
        assert np.all(np.abs(r) <= 1e-6 * (np.abs(A) @ np.abs(np.array(xh)) + np.abs(b)))
