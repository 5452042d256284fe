"""CPU oracle for the cubic grid-characteristic stage path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker.  The product (``gcm_amd``) never imports anything under ``oracle/``.

Two halves:

* ``libgcm_oracle.so`` (``gcm_oracle.c``): the per-node numerics -- matrix
  construction, Newton/min-max interpolation, ``localGcmStep`` and the stage
  loop -- restated operation by operation from the reference.
* this file: the set-up and engine semantics restated in numpy (areas,
  MaterialsCondition, InitialCondition, cubic BorderConditions, the adhesion
  ContactCopier, the AbstractEngine time loop with its Clock).  Elementwise
  numpy arithmetic on float64 is IEEE-exact, so the restatement keeps the
  reference's bits as long as each expression keeps the reference's order.

Reference files are cited as ``path:line`` relative to
``/root/reference/src/libgcm``.  Parity pins: see ``tests/test_oracle.py``.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libgcm_oracle.so")
_lib = None


def build() -> str:
    """Compile the C restatement (``oracle/Makefile``)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


class _OgGrid(ctypes.Structure):
    _fields_ = [("D", ctypes.c_int), ("M", ctypes.c_int), ("bs", ctypes.c_int),
                ("sizes", ctypes.c_int * 3), ("start", ctypes.c_int * 3),
                ("h", ctypes.c_double * 3)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        gp = ctypes.POINTER(_OgGrid)
        L.og_isotropic_elastic_matrices.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                                    ctypes.c_double, dp, dp, dp]
        L.og_interpolate.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_double, dp]
        L.og_min_max_interpolate.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_double, dp]
        L.og_diagonal_multiply.argtypes = [ctypes.c_int, dp, dp, dp]
        L.og_local_gcm_step.argtypes = [ctypes.c_int, dp, dp, dp, dp]
        L.og_interpolate_values_around.argtypes = [gp, dp, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                   dp, dp]
        L.og_stage.argtypes = [gp, ctypes.c_int, ctypes.c_double, dp, dp,
                               ctypes.POINTER(ctypes.c_uint8), dp, dp, dp, ctypes.c_int]
        L.og_fill_random.argtypes = [gp, ctypes.POINTER(ctypes.c_int), ctypes.c_uint64, dp]
        L.og_splitmix_uniform.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.og_splitmix_uniform.restype = ctypes.c_double
        L.og_size_of_all_nodes.argtypes = [gp]
        L.og_size_of_all_nodes.restype = ctypes.c_longlong
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def pde_size(D: int) -> int:
    return D + D * (D + 1) // 2


# ------------------------------------------------------------------ matrices --

def isotropic_elastic_matrices(D: int, rho: float, lam: float, mu: float):
    """ElasticModel<D>::constructGcmMatrices, identity basis
    (rheology/models/ElasticModel.hpp:57-65, 362-553).  Returns U, U1 [D,M,M], L [D,M]."""
    M = pde_size(D)
    U = np.zeros((D, M, M)); U1 = np.zeros((D, M, M)); L = np.zeros((D, M))
    if lib().og_isotropic_elastic_matrices(D, rho, lam, mu, _dp(U), _dp(U1), _dp(L)) != 0:
        raise ValueError("bad material")
    return U, U1, L


def interpolate(src: np.ndarray, q: float) -> np.ndarray:
    """EqualDistanceLineInterpolator::interpolate (interpolation/EqualDistanceLineInterpolator.hpp:56-71).
    ``src`` [n, M] is overwritten like the reference."""
    n, M = src.shape
    out = np.zeros(M)
    lib().og_interpolate(n, M, _dp(src), q, _dp(out))
    return out


def min_max_interpolate(src: np.ndarray, q: float) -> np.ndarray:
    """EqualDistanceLineInterpolator::minMaxInterpolate (hpp:18-43); raises where the reference asserts."""
    n, M = src.shape
    out = np.zeros(M)
    if lib().og_min_max_interpolate(n, M, _dp(src), q, _dp(out)) != 0:
        raise ValueError("interpolation out of range (reference assert)")
    return out


def diagonal_multiply(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    """linal::diagonalMultiply (linal/functions.hpp:254-267)."""
    M = A.shape[0]
    r = np.zeros(M)
    lib().og_diagonal_multiply(M, _dp(np.ascontiguousarray(A)), _dp(np.ascontiguousarray(B)), _dp(r))
    return r


def local_gcm_step(U1, U, V) -> np.ndarray:
    """localGcmStep (util/math/GridCharacteristicMethod.hpp:10-17)."""
    M = U.shape[0]
    out = np.zeros(M)
    lib().og_local_gcm_step(M, _dp(np.ascontiguousarray(U1)), _dp(np.ascontiguousarray(U)),
                            _dp(np.ascontiguousarray(V)), _dp(out))
    return out


def splitmix_uniform(seed: int, n: int) -> float:
    return lib().og_splitmix_uniform(seed, n)


def fill_random(body: "Body", global_sizes, seed: int):
    """Parity-random field on the inner nodes of ``body``."""
    gs = list(global_sizes) + [1] * (3 - len(global_sizes))
    lib().og_fill_random(ctypes.byref(body.g), (ctypes.c_int * 3)(*gs), seed, _dp(body.pde))


# --------------------------------------------------------------------- areas --
# util/math/Area.hpp:8-120.  An area is a tuple:
#   ("infinite",) | ("box", min3, max3) | ("sphere", radius, center3)
#   | ("cylinder", radius, begin3, end3)

def area_contains(area, X: np.ndarray, Y: np.ndarray, Z: np.ndarray) -> np.ndarray:
    kind = area[0]
    if kind == "infinite":
        return np.ones(X.shape, dtype=bool)
    if kind == "box":  # AxisAlignedBoxArea::contains (Area.hpp:37-42): open box
        mn, mx = area[1], area[2]
        ok = np.ones(X.shape, dtype=bool)
        for c, lo, hi in ((X, mn[0], mx[0]), (Y, mn[1], mx[1]), (Z, mn[2], mx[2])):
            ok &= ~((c <= lo) | (c >= hi))
        return ok
    if kind == "sphere":  # SphereArea::contains (Area.hpp:62-64): length(c - center) < r
        r, cen = area[1], area[2]
        dx = X - cen[0]; dy = Y - cen[1]; dz = Z - cen[2]
        return np.sqrt(dx * dx + dy * dy + dz * dz) < r
    if kind == "cylinder":  # StraightBoundedCylinderArea::contains (Area.hpp:91-103)
        r, b, e = area[1], np.asarray(area[2], float), np.asarray(area[3], float)
        d = e - b
        ln = math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2])
        ax = d / ln
        p0 = (X - b[0]) * ax[0] + (Y - b[1]) * ax[1] + (Z - b[2]) * ax[2]
        p1 = (X - e[0]) * ax[0] + (Y - e[1]) * ax[1] + (Z - e[2]) * ax[2]
        between = ~(p0 * p1 >= 0)
        dd = (X - b[0]) * (X - b[0]) + (Y - b[1]) * (Y - b[1]) + (Z - b[2]) * (Z - b[2])
        return between & ((dd - p0 * p0) < r * r)
    raise ValueError(kind)


# ------------------------------------------------------------------ physics --

# PhysicalQuantities::T order (util/Enum.hpp:27-50); std::map iterates by it.
QUANTITY_ORDER = ["VELOCITY", "FORCE", "Vx", "Vy", "Vz", "Sxx", "Sxy", "Sxz",
                  "Syy", "Syz", "Szz", "RHO", "PRESSURE", "DAMAGE_MEASURE"]
WAVE_COLUMN = {"P_FORWARD": 0, "P_BACKWARD": 1, "S1_FORWARD": 2, "S1_BACKWARD": 3,
               "S2_FORWARD": 4, "S2_BACKWARD": 5}  # Model.cpp:33-82 (isotropic)


def _sym_index(D, i, j):
    if i < j:
        return i * D - ((i - 1) * i) // 2 + j - i
    return j * D - ((j - 1) * j) // 2 + i - j


def quantity_index(D: int, q: str) -> Optional[int]:
    """Component index of a scalar quantity (VelocitySigmaVariables.cpp:22-66)."""
    if q in ("Vx", "Vy", "Vz"):
        i = "xyz".index(q[1])
        return i if i < D else None
    if q.startswith("S") and len(q) == 3:
        i, j = "xyz".index(q[1]), "xyz".index(q[2])
        return D + _sym_index(D, i, j) if i < D and j < D else None
    return None


def quantity_get(D: int, q: str, v: np.ndarray):
    """GetSetter::Get on PDE vectors v[..., M]."""
    if q == "PRESSURE":  # getPressure (VelocitySigmaVariables.hpp:98-104)
        tr = np.zeros(v.shape[:-1])
        for i in range(D):
            tr = tr + v[..., D + _sym_index(D, i, i)]
        return (-tr) / D
    idx = quantity_index(D, q)
    if idx is None:
        raise KeyError(q)
    return v[..., idx]


def quantity_set(D: int, q: str, value, v: np.ndarray):
    """GetSetter::Set; PRESSURE clears the whole vector (VelocitySigmaVariables.hpp:106-111)."""
    if q == "PRESSURE":
        v[...] = 0.0
        for i in range(D):
            v[..., D + _sym_index(D, i, i)] = -value
        return
    idx = quantity_index(D, q)
    if idx is None:
        raise KeyError(q)
    v[..., idx] = value


# --------------------------------------------------------------------- task --

@dataclass
class Material:
    rho: float
    lam: float
    mu: float
    tau0: float = 0.0  # IsotropicMaterial::tau0 (rheology/materials/IsotropicMaterial.hpp:17)


@dataclass
class BorderCondition:
    """Task::CubicBorderCondition (util/task/Task.hpp:185-190)."""
    direction: int
    area: tuple
    values: Dict[str, Callable[[float], float]]


@dataclass
class Task:
    """The subset of ``gcm::Task`` (util/task/Task.hpp:24-234) the cubic path reads."""
    D: int
    border_size: int
    h: Sequence[float]
    cubics: Dict[int, Tuple[Sequence[int], Sequence[int]]]  # id -> (sizes, start)
    courant: float
    default_material: Material
    inhomogeneities: List[Tuple[tuple, Material]] = field(default_factory=list)
    number_of_snaps: int = 0
    steps_per_snap: int = 1
    required_time: float = 0.0
    ic_vectors: List[Tuple[tuple, Sequence[float]]] = field(default_factory=list)
    ic_waves: List[Tuple[tuple, str, int, str, float]] = field(default_factory=list)
    ic_quantities: List[Tuple[tuple, str, float]] = field(default_factory=list)
    border_conditions: Dict[int, List[BorderCondition]] = field(default_factory=dict)
    odes: Dict[int, List[str]] = field(default_factory=dict)  # Task::Body::odes (Task.hpp:33)


class Body:
    """One cubic body: DefaultMesh storage + CubicGrid indexing (engine/cubic/DefaultMesh.hpp,
    grid/cubic/CubicGrid.hpp), restated over numpy arrays."""

    def __init__(self, task: Task, gid: int):
        sizes, start = task.cubics[gid]
        D = task.D
        self.id = gid
        self.D, self.M, self.bs = D, pde_size(D), task.border_size
        self.sizes = list(sizes) + [1] * (3 - D)
        self.start = list(start) + [0] * (3 - D)
        self.h = list(task.h) + [0.0] * (3 - D)
        if self.bs <= 0 or any(self.sizes[i] < self.bs for i in range(D)):
            raise ValueError("CubicGrid asserts sizes >= borderSize > 0 (CubicGrid.hpp:195-198)")
        self.g = _OgGrid(D, self.M, self.bs, (ctypes.c_int * 3)(*self.sizes),
                         (ctypes.c_int * 3)(*self.start), (ctypes.c_double * 3)(*self.h))
        self.shape_all = tuple(self.sizes[i] + 2 * self.bs for i in range(D))
        self.n_all = int(np.prod(self.shape_all))
        self.pde = np.zeros((self.n_all, self.M))
        self.pde_new = np.zeros((self.n_all, self.M))
        self.mat_id = np.zeros(self.n_all, dtype=np.uint8)
        self._set_up(task)

    # -- index helpers ----------------------------------------------------
    def flat_index(self, it) -> np.ndarray:
        """CubicGrid::getIndex (CubicGrid.hpp:141-147) for arrays of multi-indices [..., D]."""
        it = np.asarray(it, dtype=np.int64)
        return np.ravel_multi_index(tuple(it[..., i] + self.bs for i in range(self.D)), self.shape_all)

    def inner_indices(self) -> np.ndarray:
        """Inner multi-indices in SlowXFastZ order [N, D]."""
        grids = np.meshgrid(*[np.arange(self.sizes[i]) for i in range(self.D)], indexing="ij")
        return np.stack([g.ravel() for g in grids], axis=-1)

    def coords(self, it: np.ndarray):
        """CubicGrid::coords (CubicGrid.hpp:114-126): start*h + it*h, zero-padded to 3-D."""
        out = []
        for i in range(3):
            if i < self.D:
                out.append(float(self.start[i]) * self.h[i] + it[..., i].astype(np.float64) * self.h[i])
            else:
                out.append(np.zeros(it.shape[:-1]))
        return out

    def inner_view(self, arr=None) -> np.ndarray:
        """Inner nodes of a [n_all, M] array as an [X(,Y(,Z)), M] view."""
        a = (self.pde if arr is None else arr).reshape(self.shape_all + (self.M,))
        sl = tuple(slice(self.bs, self.bs + self.sizes[i]) for i in range(self.D))
        return a[sl]

    # -- set-up (DefaultMesh::setUpPde, DefaultMesh.hpp:60-66) -------------
    def _set_up(self, task: Task):
        D, M = self.D, self.M
        its = self.inner_indices()
        X, Y, Z = self.coords(its)
        flat = self.flat_index(its)
        # MaterialsCondition::apply (util/task/MaterialsCondition.hpp:23-36, 70-91)
        conds = [(("infinite",), task.default_material)] + list(task.inhomogeneities)
        if len(conds) > 255:
            raise ValueError("too many material conditions")
        self.tables = [isotropic_elastic_matrices(D, m.rho, m.lam, m.mu) for _, m in conds]
        self.tau0 = [m.tau0 for _, m in conds]
        self.odes = list(task.odes.get(self.id, []))
        for o in self.odes:
            if o != "MAXWELL_VISCOSITY":
                raise ValueError("only MaxwellViscosityOde compiles in the reference (Ode.hpp:50, 75)")
        mid = np.zeros(len(its), dtype=np.uint8)
        for ci, (area, _) in enumerate(conds):
            mid[area_contains(area, X, Y, Z)] = ci
        self.mat_id[flat] = mid
        # getMaximalEigenvalue (MaterialsCondition.hpp:93-101, GridCharacteristicMethod.hpp:46-61)
        ans = 0.0
        for (_, _, L) in self.tables:
            ev = 0.0
            for s in range(D):
                e = 0.0
                for k in range(M):
                    e = max(e, abs(L[s, k]))  # fmax(ans, fabs(L(i,i)))
                ev = max(ev, e)
            ans = max(ans, ev)
        self.maximal_eigenvalue = ans
        # InitialCondition::apply (util/task/InitialCondition.hpp:23-88)
        vecs = []
        for area, lst in task.ic_vectors:
            if len(lst) != M:
                raise ValueError("initial vector size")
            vecs.append((area, np.array(lst, dtype=np.float64)))
        U, U1, L = self.tables[0]  # mcConditions.front() == default material
        for area, wave_type, direction, quantity, value in task.ic_waves:
            if direction >= D:
                raise ValueError("wave direction")
            tmp = U1[direction][:, WAVE_COLUMN[wave_type]].copy()
            cur = float(quantity_get(D, quantity, tmp))
            if cur == 0:
                raise ValueError("calibration quantity is zero")
            tmp = tmp * (value / cur)
            vecs.append((area, tmp))
        for area, quantity, value in task.ic_quantities:
            tmp = np.zeros(M)
            quantity_set(D, quantity, value, tmp)
            vecs.append((area, tmp))
        acc = np.zeros((len(its), M))
        for area, v in vecs:
            m = area_contains(area, X, Y, Z)
            acc[m] = acc[m] + v
        self.pde[flat] = acc
        self._setup_borders(task)

    # -- cubic BorderConditions (engine/cubic/BorderConditions.hpp:46-114) --
    def _setup_borders(self, task: Task):
        self.border = []
        for bc in task.border_conditions.get(self.id, []):
            d = bc.direction
            for q in bc.values:
                if q != "PRESSURE" and quantity_index(self.D, q) is None:
                    raise KeyError(q)
            sides = []
            for index in (0, self.sizes[d] - 1):
                its = self.inner_indices()
                its = its[its[:, d] == index]
                X, Y, Z = self.coords(its)
                sides.append(its[area_contains(bc.area, X, Y, Z)])
            vals = sorted(bc.values.items(), key=lambda kv: QUANTITY_ORDER.index(kv[0]))
            self.border.append((d, sides[0], sides[1], vals))

    def apply_border(self, direction: int, time: float):
        for d, left, right, vals in self.border:
            if d != direction:
                continue
            for nodes, sign in ((left, 1), (right, -1)):
                if len(nodes) == 0:
                    continue
                for a in range(1, self.bs + 1):
                    inner = nodes.copy(); inner[:, d] += sign * a
                    ghost = nodes.copy(); ghost[:, d] -= sign * a
                    fi, fg = self.flat_index(inner), self.flat_index(ghost)
                    self.pde[fg] = self.pde[fi]
                    for q, f in vals:
                        inner_value = quantity_get(self.D, q, self.pde[fi])
                        ghost_value = -inner_value + 2 * f(time)
                        g = self.pde[fg]
                        quantity_set(self.D, q, ghost_value, g)
                        self.pde[fg] = g

    # -- the stage ------------------------------------------------------------
    def stage(self, s: int, tau: float, nthreads: int = 0):
        """GridCharacteristicMethod<Mesh>::stage then swapCurrAndNextPdeTimeLayer
        (engine/cubic/GridCharacteristicMethod.hpp:42-52, DefaultMesh.hpp:134-137)."""
        nm = len(self.tables)
        U = np.ascontiguousarray(np.stack([t[0] for t in self.tables]))
        U1 = np.ascontiguousarray(np.stack([t[1] for t in self.tables]))
        L = np.ascontiguousarray(np.stack([t[2] for t in self.tables]))
        mid = self.mat_id.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if nm > 1 else None
        rc = lib().og_stage(ctypes.byref(self.g), s, tau, _dp(self.pde), _dp(self.pde_new), mid,
                            _dp(U), _dp(U1), _dp(L), nthreads)
        if rc != 0:
            raise ValueError("stage: interpolation out of range (reference assert)")
        self.pde, self.pde_new = self.pde_new, self.pde

    def apply_odes(self, tau: float):
        """MaxwellViscosityOde::apply (rheology/ode/Ode.hpp:28-37) over the inner nodes:
        setSigma(getSigma() * exp(-timeStep / tau0)); the factor is the C library's exp of
        the IEEE quotient, per material (one value per node in the reference, same bits)."""
        for _ in self.odes:
            with np.errstate(divide="ignore", invalid="ignore"):
                f = [math.exp(float(np.float64(-tau) / np.float64(t0))) for t0 in self.tau0]
            flat = self.flat_index(self.inner_indices())
            fac = np.array(f)[self.mat_id[flat]]
            self.pde[flat, self.D:] = self.pde[flat, self.D:] * fac[:, None]

    def aabb(self):
        mn = np.array(self.start[:self.D])
        return mn, mn + np.array(self.sizes[:self.D]) - 1

    def box_flat(self, mn, mx_inclusive) -> np.ndarray:
        """Flat indices of a PartIterator box in SlowXFastZ order (CubicGrid.hpp:70-84)."""
        rngs = [np.arange(mn[i], mx_inclusive[i] + 1) for i in range(self.D)]
        grids = np.meshgrid(*rngs, indexing="ij")
        its = np.stack([g.ravel() for g in grids], axis=-1)
        return self.flat_index(its)


class Engine:
    """cubic::Engine<D> + AbstractEngine (engine/cubic/Engine.cpp:12-140,
    engine/AbstractEngine.cpp:9-46) without snapshotters."""

    def __init__(self, task: Task):
        self.task = task
        self.time = 0.0
        self.time_step = 0.0
        self.bodies = [Body(task, gid) for gid in sorted(task.cubics)]
        self.contacts = []  # (body, neighbour, direction, flatA, flatB)
        self._create_contacts()
        # afterConstruction (AbstractEngine.cpp:18-27)
        self.time_step = self.estimate_time_step()
        gs = task
        self.required_time = self.time_step * gs.number_of_snaps * gs.steps_per_snap
        if gs.number_of_snaps <= 0:
            self.required_time = gs.required_time
        if not self.required_time > 0:
            raise ValueError("requiredTime must be > 0")
        self.steps_done = 0

    def _create_contacts(self):
        """Engine::createGridsAndContacts (Engine.cpp:38-87)."""
        D = self.task.D
        for body in self.bodies:
            for other in self.bodies:
                if other is body:
                    continue
                amn, amx = body.aabb(); bmn, bmx = other.aabb()
                imn = np.maximum(amn, bmn); imx = np.minimum(amx, bmx)
                sizes = imx - imn
                if np.all(sizes >= 0):
                    raise ValueError("Bodies must not intersect")
                axis = 0; mw = sizes[0]
                for i in range(1, D):
                    if sizes[i] < mw:
                        axis = i; mw = sizes[i]
                if mw != -1:
                    continue
                bmin = imn.copy(); bmax = imx.copy()
                if body.start[axis] > other.start[axis]:
                    bmin[axis] -= body.bs
                else:
                    bmax[axis] += body.bs
                fa = body.box_flat(bmin - np.array(body.start[:D]), bmax - np.array(body.start[:D]))
                fb = other.box_flat(bmin - np.array(other.start[:D]), bmax - np.array(other.start[:D]))
                self.contacts.append((body, other, axis, fa, fb))

    def estimate_time_step(self) -> float:
        """Engine<D>::estimateTimeStep (Engine.cpp:124-140)."""
        mx = 0.0
        h = self.bodies[0].h
        for b in self.bodies:
            if b.maximal_eigenvalue > mx:
                mx = b.maximal_eigenvalue
        hmin = float(np.finfo(np.float64).max)
        for i in range(self.task.D):
            if hmin > h[i]:
                hmin = h[i]
        return self.task.courant * hmin / mx

    def next_time_step(self, nthreads: int = 0):
        """Engine<D>::nextTimeStep (Engine.cpp:90-121)."""
        tau = self.time_step
        for s in range(self.task.D):
            for b in self.bodies:
                b.apply_border(s, self.time)
            for body, other, axis, fa, fb in self.contacts:
                if axis == s:
                    body.pde[fa] = other.pde[fb]
            for b in self.bodies:
                b.stage(s, tau, nthreads)
        for b in self.bodies:  # Engine.cpp:115-119
            b.apply_odes(tau)

    def run(self, nthreads: int = 0, max_steps: Optional[int] = None):
        """AbstractEngine::run (AbstractEngine.cpp:30-46)."""
        while self.time < self.required_time:
            if max_steps is not None and self.steps_done >= max_steps:
                break
            self.time_step = self.estimate_time_step()
            self.next_time_step(nthreads)
            self.steps_done += 1
            self.time += self.time_step
        return self.steps_done


def step_count(time_step: float, required_time: float) -> int:
    """Number of steps AbstractEngine::run performs (Clock semantics, GlobalVariables.hpp:16-41)."""
    t, n = 0.0, 0
    while t < required_time:
        t += time_step
        n += 1
    return n
