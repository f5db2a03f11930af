#!/bin/bash
# ab_variant_build.sh NAME "FLAGS": an A/B variant of this tree in ./NAME (git-ignored, ab_* only), its native
# extension built in-tree with CANNET_EXTRA_HIPFLAGS="FLAGS" (e.g. -DCANNET_SETPRIO=1), so a GPU script can time
# `python NAME/bench.py` against `python bench.py` on one box.  The variant's object files are removed afterwards
# (only its _C travels with the gpurun snapshot).
set -euo pipefail
name=$1; flags=$2
case "$name" in ab_*) ;; *) echo "variant name must start with ab_" >&2; exit 2 ;; esac
root=$(cd "$(dirname "$0")/../.." && pwd)
cd "$root"
rm -rf "$name"
mkdir "$name"
tar --exclude=./.git --exclude=./build --exclude=./gpurun_out --exclude='./ab_*' --exclude=./profiles \
    --exclude='*.so' --exclude=__pycache__ -cf - . | tar -xf - -C "$name"
(cd "$name" && CANNET_EXTRA_HIPFLAGS="$flags" python -c "
import sys; sys.path.insert(0, '.')
from can_distributed_pytorch_amd import build_native as b
b.build(jobs=8)
print('built', b.ext_path())")
rm -rf "$name/build"
