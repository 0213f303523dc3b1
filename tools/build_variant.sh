#!/bin/bash
# Build an A/B variant of libclvmcmc.so with extra compile flags for kernels.hip and capi.hip:
#   tools/build_variant.sh NAME "-DKNOB=VALUE ..."   ->  build/NAME/libclvmcmc.so
# (run bench/tests against it with CLV_LIB_PATH=build/NAME/libclvmcmc.so).  The other objects are
# the in-tree ones (make first).
set -e
R=$(cd "$(dirname "$0")/.." && pwd); C=$R/mcmc_clv_model_amd/csrc
mkdir -p $R/build/$1
# a third argument "capi": the flags only change host code — kernels.o is the in-tree one
if [ "$3" = capi ]; then cp $C/kernels.o $R/build/$1/kernels.o; else
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-bitwise-instead-of-logical \
  -ffp-contract=off $2 -c $C/kernels.hip -o $R/build/$1/kernels.o
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable -Wno-bitwise-instead-of-logical \
  -ffp-contract=off $2 -c $C/capi.hip -o $R/build/$1/capi.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $R/build/$1/kernels.o $R/build/$1/capi.o $C/analysis.o $C/elog.o $C/group.o \
  $C/drawstream.o $C/probe.o -lpthread -o $R/build/$1/libclvmcmc.so
echo built build/$1/libclvmcmc.so
