cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for S in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams $S > gpurun_out/s$S.log 2>&1 || exit $?
  echo "S=$S $(grep -o '"value": [0-9.]*' gpurun_out/s$S.log) $(grep -o '"walk_kernel": {"avg_ms": [0-9.]*' gpurun_out/s$S.log) $(grep -o '"events_kernel": {"avg_ms": [0-9.]*' gpurun_out/s$S.log)" | tee -a gpurun_out/s12.txt
done; done
for b in 8 16; do for S in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --streams $S --batches $b > gpurun_out/sb.log 2>&1 || exit $?
  echo "batches=$b S=$S $(grep -o '"value": [0-9.]*' gpurun_out/sb.log)" | tee -a gpurun_out/s12.txt
done; done
