export TMPDIR=/tmp; mkdir -p gpurun_out/prof_train
timeout -k 10 200 python tools/probes/train_trace.py > gpurun_out/prof_train/plain.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train/trace -o run --output-format csv -- python3 tools/probes/train_trace.py > gpurun_out/prof_train/log.txt 2>&1
cat gpurun_out/prof_train/plain.txt
