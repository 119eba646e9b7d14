#!/bin/bash
# The routed shard path on hardware (run via gpurun):  bash tools/rccl_trace.sh TAG
# rocprofv3 kernel trace of tests/test_gpu_shard.py's forced-route case
# (tools/rccl_routed.py: the same worker, in one process) at
# world 1 over RCCL (shm__shard_force_route: the rank's own requests go
# through ncclSend/ncclRecv to itself), so the trace shows the exchange's
# RCCL kernels between the route and walk kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
OUT=$R/gpurun_out/rccl_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/rccl_routed.py > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
grep -i "nccl\|rccl" $OUT/trace/run_kernel_stats.csv | cut -c1-160 || true
echo rccl_trace done
