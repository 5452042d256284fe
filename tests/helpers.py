"""Shared test helpers: build matching oracle bodies and gcmx contexts."""
import numpy as np

from oracle import oracle as O


def oracle_body(D, bs, sizes, start=None, h=None, materials=((4.0, 2.0, 1.0),), courant=0.9):
    """An oracle Body with zero state (no initial conditions)."""
    start = list(start) if start is not None else [0] * D
    h = list(h) if h is not None else [1.0] * D
    mats = [O.Material(*m) for m in materials]
    inh = [(("infinite",), m) for m in mats[1:]]
    t = O.Task(D=D, border_size=bs, h=h, cubics={0: (list(sizes), start)}, courant=courant,
               default_material=mats[0], inhomogeneities=inh, number_of_snaps=1)
    return O.Engine(t).bodies[0]


def random_state(body, seed, ghosts=True):
    rng = np.random.default_rng(seed)
    if ghosts:
        body.pde[:] = rng.uniform(-1, 1, body.pde.shape)
    else:
        body.pde[:] = 0.0
        body.inner_view()[...] = rng.uniform(-1, 1, body.inner_view().shape)


def random_materials(body, seed):
    """Random per-node material ids over the inner nodes (ghosts keep 0)."""
    rng = np.random.default_rng(seed)
    its = body.inner_indices()
    body.mat_id[body.flat_index(its)] = rng.integers(0, len(body.tables), len(its)).astype(np.uint8)


def tables(body):
    U = np.stack([t[0] for t in body.tables]); U1 = np.stack([t[1] for t in body.tables])
    L = np.stack([t[2] for t in body.tables])
    return U, U1, L


def context_for(body, path=None, device=0):
    import gcm_amd
    ctx = gcm_amd.Context(body.D, body.bs, body.sizes[:body.D], start=body.start[:body.D],
                          h=body.h[:body.D], device=device)
    U, U1, L = tables(body)
    ctx.set_materials(U, U1, L)
    if len(body.tables) > 1:
        ctx.set_material_ids(body.mat_id)
    ctx.upload(body.pde)
    if path is not None:
        ctx.set_path(path)
    return ctx


def assert_same(ctx, body, what=""):
    got = ctx.download()
    want = body.pde
    if not np.array_equal(got, want):
        diff = got != want
        idx = np.argwhere(diff)
        n = int(diff.sum())
        i0 = tuple(idx[0])
        raise AssertionError(f"{what}: {n} values differ; first at {i0}: "
                             f"got {got[i0]!r} want {want[i0]!r}")


def assert_same_inner(ctx, body, what=""):
    """Inner nodes only: the one-pass face step (gcmx_step_faces) forms the ghost
    rows / columns of the intermediate stages in registers and LDS, so the ghost
    memory of the layers is not part of its state (every ghost a stage reads is
    refilled before that stage, as in the reference)."""
    got = body.inner_view(ctx.download().reshape(body.pde.shape))
    want = body.inner_view(body.pde)
    if not np.array_equal(got, want):
        diff = got != want
        idx = np.argwhere(diff)
        raise AssertionError(f"{what}: {int(diff.sum())} inner values differ; first at "
                             f"{tuple(idx[0])}: got {got[tuple(idx[0])]!r} want {want[tuple(idx[0])]!r}")


def seq_sum(a):
    s = 0.0
    for x in np.asarray(a).reshape(-1).tolist():
        s += x
    return s


def read_vts(path):
    """Parse a VTK XML StructuredGrid file with appended raw data (UInt64 headers,
    Float32 arrays) as gcm_amd's VtkSnapshotter writes it.  Returns
    (dims, {name: array [n, components]}, points [n, 3]); points in VTK order."""
    import re
    raw = open(path, "rb").read()
    head, _, rest = raw.partition(b"<AppendedData encoding=\"raw\">")
    text = head.decode()
    m = re.search(r'WholeExtent="([^"]+)"', text)
    ext = [int(v) for v in m.group(1).split()]
    dims = (ext[1] + 1, ext[3] + 1, ext[5] + 1)
    data = rest[rest.index(b"_") + 1:]
    arrays = {}
    for name, comps, off in re.findall(
            r'<DataArray type="Float32" Name="([^"]+)" NumberOfComponents="(\d+)" '
            r'format="appended" offset="(\d+)"/>', text):
        off = int(off)
        nbytes = int(np.frombuffer(data[off:off + 8], dtype="<u8")[0])
        arrays[name] = np.frombuffer(data[off + 8:off + 8 + nbytes], dtype="<f4").reshape(-1, int(comps))
    points = arrays.pop("Points")
    return dims, arrays, points


def read_vtu(path):
    """Parse a VTK XML UnstructuredGrid file with appended raw data (UInt64 headers)
    as gcm_amd's simplex VtkSnapshotter writes it.  Returns ({name: array [n, c]},
    points [n, 3], connectivity [m, 4], offsets [m], types [m])."""
    import re
    raw = open(path, "rb").read()
    head, _, rest = raw.partition(b"<AppendedData encoding=\"raw\">")
    text = head.decode()
    data = rest[rest.index(b"_") + 1:]
    dt = {"Float32": "<f4", "Int64": "<i8", "UInt8": "u1"}
    arrays = {}
    for typ, name, tail in re.findall(r'<DataArray type="(\w+)" Name="([^"]+)"([^/]*)/>', text):
        off = int(re.search(r'offset="(\d+)"', tail).group(1))
        comps = re.search(r'NumberOfComponents="(\d+)"', tail)
        nbytes = int(np.frombuffer(data[off:off + 8], dtype="<u8")[0])
        a = np.frombuffer(data[off + 8:off + 8 + nbytes], dtype=dt[typ])
        arrays[name] = a.reshape(-1, int(comps.group(1))) if comps else a
    points = arrays.pop("Points")
    conn = arrays.pop("connectivity").reshape(-1, 4)
    return arrays, points, conn, arrays.pop("offsets"), arrays.pop("types")
