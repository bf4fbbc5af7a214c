cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for b in 64 32 16 8; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --batches $b > gpurun_out/strong_$b.log 2>&1 || exit $?
  echo "batches=$b $(grep -o '"value": [0-9.]*' gpurun_out/strong_$b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/strong_$b.log) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/strong_$b.log)" | tee -a gpurun_out/strong.txt
done
