#!/bin/bash
# fused decode v2 probes on the probe library (make -C clay_amd/csrc probe): the 4-erasure
# (10,4,13) 1 GiB decode under CLAY_DECODE_PROBE = each of $PROBES (0 = plain; 40 s_memtime
# segments; 41 rounds at priority 0; 42 = 41 with segments; 31/32/34/35 parts switched off).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-f2p}
for pr in ${PROBES:-0 40 41 42}; do
  CLAY_AMD_LIB=$R/clay_amd/libclay_amd_probe.so CLAY_EXEC=stream-fused2 CLAY_DECODE_PROBE=$pr ONLY=cfg5 RUNS=${RUNS:-10} timeout -k 10 120 python scripts/bench_paths.py > gpurun_out/${TAG}_p$pr.jsonl 2> gpurun_out/${TAG}_p$pr.err || { echo "probe $pr failed"; tail -5 gpurun_out/${TAG}_p$pr.err; exit 1; }
  echo "probe $pr"; grep -h "0, 4, 8, 12\|f2-timing" gpurun_out/${TAG}_p$pr.jsonl | head -8
done
