#!/bin/bash
# Kernel trace + PMC passes (one counter group per rocprofv3 run, --pmc only) of the (10,4,13)
# 1 GiB decode of erasures $ER (default 0,4,8,12) on exec mode $CLAY_EXEC (default auto):
# HBM bytes (FETCH_SIZE / WRITE_SIZE) and the SQ instruction mix, for scripts/pmc_summary.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-pmcd}
ER=${ER:-0,4,8,12}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/trace" -o p -- python3 "$R/scripts/prof_decode.py" --er $ER --iters 20 > "$R/gpurun_out/$TAG/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/$TAG/trace.log"; exit 1; }
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$TAG/$n" -o p -- python3 "$R/scripts/prof_decode.py" --er $ER --iters 4 > "$R/gpurun_out/$TAG/$n.log" 2>&1 || { echo "pmc $n failed"; tail -5 "$R/gpurun_out/$TAG/$n.log"; exit 1; }
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES && \
echo "pmc done" && find "$R/gpurun_out/$TAG" -name "*kernel_stats*"
