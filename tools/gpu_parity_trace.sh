set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; tail -3 gpurun_out/parity.log; [ $rc -ne 0 ] && exit $rc
bash tools/trace_quick.sh r02b
