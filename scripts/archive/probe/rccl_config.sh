# RCCL communicator config probe (one rank): which minCTAs / maxCTAs this
# box's RCCL accepts (gcmx_comm_init, ncclCommInitRankConfig).
cd "${GRAFT_REPO_ROOT}"
for M in "0 0" "16 32" "16 64" "32 64" "64 128"; do
  set -- $M
  echo "== min ctas $1 max $2"
  GCMX_COMM_MIN_CTAS=$1 GCMX_COMM_MAX_CTAS=$2 NCCL_DEBUG=WARN timeout -k 5 60 python -c "
import gcm_amd
from gcm_amd.host import isotropic_elastic_matrices
U,U1,L = isotropic_elastic_matrices(3,4,2,1)
c = gcm_amd.Context(3,2,[16,24,64]); c.set_materials(U[None],U1[None],L[None])
try:
    c.comm_init(gcm_amd.unique_id(),1,0,-1,-1); c.step(0.9); c.sync(); print('ok')
except Exception as e: print('ERR', e)
" 2>&1 | grep -v "amdgpu.ids\|alt_rsmi\|^$" | tail -3
done
