# Tuning builds of the library into build/ (never the product; select one with
# MGMC_LIBRARY=build/libmgmc_<name>.so).  Every knob here is a bitwise-neutral tunable (tile shapes,
# chunk depths, launch thresholds): results equal the product's, only the speed differs.  Timing
# decompositions that change results (round 1-2's MGMC_*_EXP switches) are no longer in the product
# sources.
cd "$(dirname "$0")/../multigridmc_amd/csrc" && mkdir -p ../../build
HIPX="/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -w --offload-arch=gfx950 -shared"
SRCS="mgmc_capi.hip mgmc_hierarchy.cpp mgmc_operators.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib"
# fine-sweep tile shapes TYxMINW[xTZ[xTYPxMINWP]] (rows per tile, waves/SIMD floor, z-chunk, then
# the same for the fused-prolongation sweep; 32 x-pairs): build/libmgmc_exps<shape>.so
for s in ${SHAPES:-}; do
  IFS=x read -r ty mw tz typ mwp <<< "$s"
  d="-DMGMC_ZS_SHAPE_TY=$ty -DMGMC_ZS_SHAPE_MINW=$mw ${tz:+-DMGMC_ZS_SHAPE_TZ=$tz}"
  d="$d ${typ:+-DMGMC_ZS_SHAPE_TYP=$typ -DMGMC_ZS_SHAPE_MINWP=$mwp}"
  $HIPX $d -o ../../build/libmgmc_exps$s.so $SRCS &
done
# fused-prolongation sweep z-chunk depths: build/libmgmc_expz<TZP>.so
for z in ${TZPS:-}; do
  $HIPX -DMGMC_ZS_SHAPE_TZP=$z -o ../../build/libmgmc_expz$z.so $SRCS &
done
# quad passes on 3D levels with rows of up to QMAX pairs (build/libmgmc_expm<QMAX>.so)
for q in ${QMAX:-}; do
  IFS=x read -r mp nt <<< "$q"
  $HIPX -DMGMC_QUADS_MAXPAIR=$mp ${nt:+-DMGMC_QUADS_NT=$nt} -o ../../build/libmgmc_expm$q.so $SRCS &
done
# low-rank dots: the staged kernel below LRSW wavefronts of the per-block kernel (build/libmgmc_expw<N>.so)
for w in ${LRSW:-}; do
  $HIPX -DLRS_MAX_WAVES=$w -o ../../build/libmgmc_expw$w.so $SRCS &
done
# free-form variants NAME=defines (build/libmgmc_<NAME>.so), e.g. VARIANTS="a=-DMGMC_X=1 b=-DMGMC_X=2"
for v in ${VARIANTS:-}; do
  name=${v%%=*}; defs=${v#*=}
  $HIPX ${defs//,/ } -o ../../build/libmgmc_$name.so $SRCS &
done
wait
