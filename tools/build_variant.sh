#!/bin/bash
# Build a variant of the verifier library for in-process A/B timing (tools/ab.py).
# usage: tools/build_variant.sh NAME [hipcc -D flags...]   -> build/ab/libpbft_NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ab
name=$1; shift
python3 - "$name" "$@" <<'PY'
import sys
sys.path.insert(0, ".")
from pbft_amd import native_build
name, defines = sys.argv[1], sys.argv[2:]
native_build.build_library(f"build/ab/libpbft_{name}.so", defines, objdir=f"build/ab/obj_{name}")
PY
echo built build/ab/libpbft_$name.so
