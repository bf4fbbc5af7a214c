#!/bin/bash
# tools/ab_enc.sh <name> [hipcc flags...]: tempme_amd/lib/ab/<name>.so = the in-tree objects (make first) with
# encoder.hip recompiled under the given flags (walk_kernel build variants; faster than tools/ab_build.sh)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
make -s -C tempme_amd/csrc
mkdir -p tempme_amd/lib/ab /tmp/ab_enc
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -Wno-unused-result -Iinclude"
/opt/rocm/bin/hipcc $F "$@" -x hip -c tempme_amd/csrc/encoder.hip -o /tmp/ab_enc/$name.o
objs=$(ls tempme_amd/lib/obj/*.o | grep -v '/encoder.hip.o$')
/opt/rocm/bin/hipcc $F -shared -o tempme_amd/lib/ab/$name.so /tmp/ab_enc/$name.o $objs
echo "built tempme_amd/lib/ab/$name.so"
