export TMPDIR=/tmp
timeout -k 10 200 python3 tools/probes/wave_timeline.py synthetic > gpurun_out/tl_syn.log 2>&1 && timeout -k 10 200 python3 tools/probes/wave_timeline.py train_like > gpurun_out/tl_tl.log 2>&1
rc=$?; cat gpurun_out/tl_syn.log gpurun_out/tl_tl.log | grep -v amdgpu.ids; exit $rc
