# Timing-experiment builds of the library (MGMC_ZS_EXP=1..4, see mgmc_zsweep.hpp) into build/.
# Never loaded by the product; select one with MGMC_LIBRARY=build/libmgmc_exp<N>.so.
cd "$(dirname "$0")/../multigridmc_amd/csrc" && mkdir -p ../../build
HIPX="/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -w --offload-arch=gfx950 -shared"
SRCS="mgmc_capi.hip mgmc_hierarchy.cpp mgmc_operators.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib"
for n in ${EXPS:-1 2 3 4}; do
  $HIPX -DMGMC_ZS_EXP=$n -o ../../build/libmgmc_exp$n.so $SRCS &
done
# cache-policy variants: 7 non-temporal stores, 8 non-temporal f loads, 9 both
for n in ${NTEXPS:-}; do
  d="-DMGMC_ZS_NT_STORE=$(( n == 7 || n == 9 )) -DMGMC_ZS_NT_F=$(( n == 8 || n == 9 ))"
  $HIPX $d -o ../../build/libmgmc_exp$n.so $SRCS &
done
# fine-sweep tile shapes XPxTYxNT[xTZ] (x-pairs, rows, threads, z-chunk): build/libmgmc_exps<shape>.so
for s in ${SHAPES:-}; do
  IFS=x read -r xp ty nt tz <<< "$s"
  d="-DMGMC_ZS_SHAPE_XP=$xp -DMGMC_ZS_SHAPE_TY=$ty -DMGMC_ZS_SHAPE_NT=$nt ${tz:+-DMGMC_ZS_SHAPE_TZ=$tz}"
  $HIPX $d -o ../../build/libmgmc_exps$s.so $SRCS &
done
wait
