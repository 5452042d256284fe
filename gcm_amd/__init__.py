"""gcm_amd -- MI355X-native grid-characteristic elastic-wave stepper.

The hot path (libgcm's cubic stage loop) lives in ``lib/libgcmx.so``: hand-written
gfx950 HIP kernels behind the C-ABI declared in ``include/gcmx.h``.  This package
holds the Python side of that boundary (``gcm_amd.gcmx``) and the host mirror of
the reference's Engine / Task / factory surface, the C++ engine of ``host/``
bound as ``gcm_amd._gcm_host``.
"""
from .gcmx import (Context, FP_EXACT, FP_FMA, GcmxError, LIB_PATH, PATH_AUTO, PATH_FUSED, PATH_GENERIC,
                   PATH_SPLIT, SCHED_AUTO, SCHED_BFIRST, SCHED_SINGLE, SCHED_XSLAB, comm_init_local, lib,
                   local_group_steps, pde_size, unique_id)

__all__ = ["Context", "FP_EXACT", "FP_FMA", "GcmxError", "LIB_PATH", "PATH_AUTO", "PATH_FUSED", "PATH_GENERIC",
           "PATH_SPLIT", "SCHED_AUTO", "SCHED_BFIRST", "SCHED_SINGLE", "SCHED_XSLAB", "comm_init_local", "lib",
           "local_group_steps", "pde_size", "unique_id"]
