#!/bin/bash
# Round 6, first GPU call: the new GPU tests (capture-open release, codeword exec-mode gating,
# misaligned local256 pointers), the live-math encode breakdown (stream_probe v), one PMC pass of
# SQ_INSTS_VALU per variant (stream_probe w), and last the bounds-checked no-barrier timing probe
# (stream_probe f).  Every GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06a}
cd "$R"
echo "[$(date +%T)] pytest (new tests)"
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  "tests/test_gpu_runtime.py::test_release_captured_refused_while_capture_open" \
  "tests/test_gpu_codeword_decode.py" \
  "tests/test_gpu_stream_local.py::test_local256_misaligned_chunk_pointers" \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
echo "[$(date +%T)] stream_probe v"
timeout -k 10 240 ./bench_tools/stream_probe 419432 v > gpurun_out/${TAG}_variants.txt 2>&1 || { echo "probe v failed rc=$?"; tail -20 gpurun_out/${TAG}_variants.txt; exit 1; }
cat gpurun_out/${TAG}_variants.txt
echo "[$(date +%T)] stream_probe n (round-6 lane map A/B)"
timeout -k 10 240 ./bench_tools/stream_probe 419432 n > gpurun_out/${TAG}_map.txt 2>&1 || { echo "probe n failed rc=$?"; tail -20 gpurun_out/${TAG}_map.txt; exit 1; }
cat gpurun_out/${TAG}_map.txt
echo "[$(date +%T)] rocprofv3 pmc SQ_INSTS_VALU"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d "$R/gpurun_out/${TAG}_pmc" -o valu -- "$R/bench_tools/stream_probe" 419432 w > "$R/gpurun_out/${TAG}_pmc.txt" 2>&1 || { echo "pmc failed rc=$?"; tail -20 "$R/gpurun_out/${TAG}_pmc.txt"; exit 1; }
cd "$R"
echo "[$(date +%T)] stream_probe f (bounds-checked no-barrier timing probe)"
timeout -k 10 120 ./bench_tools/stream_probe 419432 f > gpurun_out/${TAG}_fault.txt 2>&1 || { echo "probe f failed rc=$?"; tail -20 gpurun_out/${TAG}_fault.txt; exit 1; }
cat gpurun_out/${TAG}_fault.txt
echo "[$(date +%T)] done"
