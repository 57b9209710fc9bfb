#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only) for one encode path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; PATHSEL=$2; TILE=${3:-0}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
cd /tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/$TAG/$n" -o p -- python3 "$R/scripts/prof_encode.py" --path $PATHSEL --tile $TILE --iters 4 > "$R/gpurun_out/$TAG/$n.log" 2>&1
}
run sq  SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU && \
run ta  TA_TA_BUSY GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES && \
run ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_SALU SQ_INSTS_SMEM
