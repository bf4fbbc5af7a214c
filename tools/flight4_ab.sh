cd "${GRAFT_REPO_ROOT}" && export TMPDIR=/tmp
for r in 1 2; do for st in 3 4; do for b in 24 48; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras --batches $b --streams $st --overlap-walk > gpurun_out/s4_${st}_${b}_$r.log 2>&1 || exit $?
  echo "streams=$st b=$b r=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s4_${st}_${b}_$r.log | head -1)" | tee -a gpurun_out/s4.txt
done; done; done
