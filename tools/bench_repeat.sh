set -o pipefail
O=gpurun_out/rep; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/b_$i.log 2>&1 || exit 1
  grep "^{" $O/b_$i.log | tail -1 | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); t=j['train_step']; print(j['value'], t['ms'], t['bf16_mlp']['ms'])"
done
