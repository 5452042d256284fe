"""Python access to the C++ host mirror (gcm_amd/host, lib/libgcm_host.so)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB_PATH = os.path.join(_HERE, "lib", "libgcm_host.so")
_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(HOST_LIB_PATH):
            raise ImportError(f"{HOST_LIB_PATH} not built: run __graft_entry__.build()")
        L = ctypes.CDLL(HOST_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        L.gcm_host_isotropic_elastic_matrices.argtypes = [ctypes.c_int, ctypes.c_double,
                                                          ctypes.c_double, ctypes.c_double,
                                                          dp, dp, dp]
        _lib = L
    return _lib


def isotropic_elastic_matrices(D: int, rho: float, lam: float, mu: float):
    """ElasticModel<D>::constructGcmMatrices (identity basis): U, U1 [D,M,M], L [D,M]."""
    M = D + D * (D + 1) // 2
    U = np.zeros((D, M, M)); U1 = np.zeros((D, M, M)); L = np.zeros((D, M))
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    if lib().gcm_host_isotropic_elastic_matrices(D, rho, lam, mu, dp(U), dp(U1), dp(L)) != 0:
        raise ValueError("bad isotropic material (needs rho > 0, mu > 0)")
    return U, U1, L
