#!/bin/bash
# tools/gpurun_retry.sh <out> <cmd>: retry a gpurun call only while the pool reports no free slot/box (nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 30); do
  timeout 1500 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "$out" 2>&1
  if grep -q "nothing was charged\|no free box right now\|backing off\|stopped responding while being prepared" "$out" && ! grep -q "^=== " "$out"; then
    echo "transient (attempt $i)" >> "$out.tries"; sleep 150; continue
  fi
  break
done
echo done >> "$out"
