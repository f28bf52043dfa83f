export TMPDIR=/tmp
mkdir -p gpurun_out/hb
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/hb/tests.log 2>&1
rc=$?; tail -3 gpurun_out/hb/tests.log; [ $rc -ne 0 ] && exit $rc
DTYPES=fp32 TAG=hb bash tools/train_prof.sh
