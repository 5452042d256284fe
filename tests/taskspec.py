"""One task description, two builders: the oracle's Task and the product's
C++ host Task (gcm_amd._gcm_host).  Field names follow gcm::Task."""
from oracle import oracle as O


def spec(D, bs, h, cubics, courant, material, inhomogeneities=(), snaps=0, steps_per_snap=1,
         required_time=0.0, vectors=(), waves=(), quantities=(), borders=None, odes=None):
    """material tuples: (rho, lambda, mu[, tau0]); odes: {body: ["MAXWELL_VISCOSITY", ..]}."""
    return dict(D=D, bs=bs, h=list(h), cubics=dict(cubics), courant=courant, material=material,
                inhomogeneities=list(inhomogeneities), snaps=snaps, steps_per_snap=steps_per_snap,
                required_time=required_time, vectors=list(vectors), waves=list(waves),
                quantities=list(quantities), borders=borders or {}, odes=odes or {})


def oracle_task(s):
    return O.Task(D=s["D"], border_size=s["bs"], h=s["h"], cubics=s["cubics"], courant=s["courant"],
                  default_material=O.Material(*s["material"]),
                  inhomogeneities=[(a, O.Material(*m)) for a, m in s["inhomogeneities"]],
                  number_of_snaps=s["snaps"], steps_per_snap=s["steps_per_snap"],
                  required_time=s["required_time"], ic_vectors=s["vectors"], ic_waves=s["waves"],
                  ic_quantities=s["quantities"],
                  border_conditions={b: [O.BorderCondition(d, a, v) for d, a, v in lst]
                                     for b, lst in s["borders"].items()},
                  odes={b: list(v) for b, v in s["odes"].items()})


def host_task(s):
    from gcm_amd import _gcm_host as H
    t = H.Task()
    t.dimensionality = s["D"]
    t.border_size = s["bs"]
    t.h = s["h"]
    t.courant = s["courant"]
    t.number_of_snaps = s["snaps"]
    t.steps_per_snap = s["steps_per_snap"]
    t.required_time = s["required_time"]
    for gid, (sizes, start) in s["cubics"].items():
        t.add_body(gid, list(sizes), list(start))
    t.set_default_material(*s["material"])
    for a, m in s["inhomogeneities"]:
        t.add_material(a, *m)
    for a, v in s["vectors"]:
        t.add_initial_vector(a, list(v))
    for a, w, d, q, val in s["waves"]:
        t.add_initial_wave(a, w, d, q, val)
    for a, q, val in s["quantities"]:
        t.add_initial_quantity(a, q, val)
    for b, lst in s["borders"].items():
        for d, a, v in lst:
            t.add_border_condition(b, d, a, v)
    for b, lst in s["odes"].items():
        for o in lst:
            t.add_ode(b, o)
    return t
