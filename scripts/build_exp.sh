# Timing-experiment builds of the library (MGMC_ZS_EXP=1..4, see mgmc_zsweep.hpp) into build/.
# Never loaded by the product; select one with MGMC_LIBRARY=build/libmgmc_exp<N>.so.
cd "$(dirname "$0")/../multigridmc_amd/csrc" && mkdir -p ../../build
for n in ${EXPS:-1 2 3 4}; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -w --offload-arch=gfx950 -DMGMC_ZS_EXP=$n -shared \
    -o ../../build/libmgmc_exp$n.so mgmc_capi.hip mgmc_hierarchy.cpp mgmc_operators.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
# cache-policy variants: 7 non-temporal stores, 8 non-temporal f loads, 9 both
for n in ${NTEXPS:-}; do
  d="-DMGMC_ZS_NT_STORE=$(( n == 7 || n == 9 )) -DMGMC_ZS_NT_F=$(( n == 8 || n == 9 ))"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -w --offload-arch=gfx950 $d -shared \
    -o ../../build/libmgmc_exp$n.so mgmc_capi.hip mgmc_hierarchy.cpp mgmc_operators.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done

wait
