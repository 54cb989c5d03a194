#!/bin/bash
# Build a variant of the verifier library for in-process A/B timing (tools/ab.py).
# usage: tools/build_variant.sh NAME [hipcc -D flags...]   -> build/ab/libpbft_NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ab
name=$1; shift
for h in replica wire; do
  [ build/$h.o -nt pbft_amd/csrc/host/$h.cpp ] || g++ -O2 -std=c++17 -fPIC -c -o build/$h.o pbft_amd/csrc/host/$h.cpp
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" -o build/ab/libpbft_$name.so \
  pbft_amd/csrc/pbft_verify.hip -x none build/replica.o build/wire.o
echo built build/ab/libpbft_$name.so
