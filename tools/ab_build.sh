#!/bin/bash
# tools/ab_build.sh <name> <encoder.hip>: build tempme_amd/lib/ab/<name>.so from the current sources
# with encoder.hip replaced by the given file (A/B timing of walk_kernel variants on one box);
# SAMPLER=<file> / TRAIN=<file> / GM=<file> / TGN=<file> replace sampler.hip / encoder_train.hip / graphmixer.hip /
# tgn_attn.hip the same way.
set -e
cd "$(dirname "$0")/.."
name=$1; enc=$2
out=ab_src/$name; mkdir -p "$out" tempme_amd/lib/ab
cp tempme_amd/csrc/*.h tempme_amd/csrc/*.cpp tempme_amd/csrc/*.hip "$out/"
rm -f "$out/dropin_ext.cpp"   # the torch host extension, not part of the library
cp "$enc" "$out/encoder.hip"
[ -n "$SAMPLER" ] && cp "$SAMPLER" "$out/sampler.hip"
[ -n "$TRAIN" ] && cp "$TRAIN" "$out/encoder_train.hip"
[ -n "$GM" ] && cp "$GM" "$out/graphmixer.hip"
[ -n "$TGN" ] && cp "$TGN" "$out/tgn_attn.hip"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -Wno-unused-result -Iinclude $EXTRA"
pids=()
for s in $(cd "$out" && ls *.cpp *.hip); do /opt/rocm/bin/hipcc $F -x hip -c "$out/$s" -o "$out/$s.o" & pids+=($!); done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed"; rm -rf "$out"; exit 1; }; done
/opt/rocm/bin/hipcc $F -shared -o "tempme_amd/lib/ab/$name.so" "$out"/*.o
rm -rf "$out"; rmdir ab_src 2>/dev/null || true
echo "built tempme_amd/lib/ab/$name.so"
