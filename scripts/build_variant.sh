#!/bin/bash
# Build an experiment variant of libspt_hip.so with extra -D flags on the kernels:
#   scripts/build_variant.sh NAME "-DFOO=1 ..."   ->  build/libspt_exp_NAME.so  (use with SPT_LIB_PATH)
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
# parity-breaking measurement flags (spt_device.h SPT_EXPERIMENT_*) compile only with this explicit define
case "$flags" in *SPT_EXPERIMENT_*) flags="$flags -DSPT_EXPERIMENT_BUILD" ;; esac
mkdir -p build/var_$name
H="/opt/rocm/bin/hipcc -O3 -fno-slp-vectorize -ffp-contract=off -fno-fast-math -fPIC -std=c++17 --offload-arch=gfx950 -fno-gpu-rdc -Iinclude -Isoftware-path-tracer_amd/csrc"
$H $flags -c software-path-tracer_amd/csrc/spt_kernels.hip -o build/var_$name/k.o
$H $flags -c software-path-tracer_amd/csrc/spt_capi.hip -o build/var_$name/c.o
# the run-time specialized kernels compile the variant's own kernel source, not the in-tree build's
C=software-path-tracer_amd/csrc
python3 scripts/embed_sources.py build/var_$name/spt_jit_src.inc $C/spt_kernels.hip $C/spt_device.h $C/spt_kernels.h
$H $flags "-DSPT_JIT_EXTRA_OPTS=\"$flags\"" -Ibuild/var_$name -c software-path-tracer_amd/csrc/spt_jit.hip -o build/var_$name/j.o
# the host scene preparation (BVH build, collapse, node order) takes the variant's flags too
g++ -O2 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Iinclude -I$C $flags -c $C/scene.cpp -o build/var_$name/s.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fno-gpu-rdc -o build/libspt_exp_$name.so build/var_$name/k.o build/var_$name/c.o build/var_$name/j.o \
  build/var_$name/s.o software-path-tracer_amd/build/scenes.o
echo build/libspt_exp_$name.so
