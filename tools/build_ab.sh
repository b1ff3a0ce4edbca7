#!/bin/bash
# Build an A/B copy of libqpp.so with extra hipcc flags: tools/build_ab.sh <name> [flags...] -> ab/<name>.so
set -e
name=$1; shift
root=$(cd $(dirname $0)/.. && pwd)
src=$root/s2n-quic_amd/csrc
out=$root/ab; tmp=$(mktemp -d)
mkdir -p $out
pids=()
for f in aes_gcm.hip quad.hip burst.hip chacha.hip plan.hip keysched.hip fips.hip api.cpp kdf.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value --offload-arch=${ARCH:-gfx950} -munsafe-fp-atomics "$@" -c $src/$f -o $tmp/${f%.*}.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "compile failed (pid $p)"; rm -rf $tmp; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=${ARCH:-gfx950} -shared -fPIC -o $out/$name.so $tmp/*.o -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined
rm -rf $tmp
echo "built ab/$name.so"
