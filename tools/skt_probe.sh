export TMPDIR=/tmp
mkdir -p gpurun_out/skt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/skt/trace -o run --output-format csv -- python3 tools/probes/small_kernels_time.py > gpurun_out/skt/log.txt 2>&1 && cat gpurun_out/skt/log.txt && python3 tools/kstats.py gpurun_out/skt/trace 13 12
