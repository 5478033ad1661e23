# Timing-experiment builds of the library (MGMC_ZS_EXP=1..4, see mgmc_zsweep.hpp) into build/.
# Never loaded by the product; select one with MGMC_LIBRARY=build/libmgmc_exp<N>.so.
cd "$(dirname "$0")/../multigridmc_amd/csrc" && mkdir -p ../../build
HIPX="/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -w --offload-arch=gfx950 -shared"
SRCS="mgmc_capi.hip mgmc_hierarchy.cpp mgmc_operators.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib"
for n in ${EXPS:-1 2 3 4}; do  # MGMC_ZS_EXP variants
  $HIPX -DMGMC_ZS_EXP=$n -o ../../build/libmgmc_exp$n.so $SRCS &
done
# cache-policy variant 7: plain (temporal) sweep stores
for n in ${NTEXPS:-}; do
  $HIPX -DMGMC_ZS_NT_STORE=0 -o ../../build/libmgmc_exp$n.so $SRCS &
done
# fine-sweep tile shapes TYxMINW[xTZ[xTYPxMINWP]] (rows per tile, waves/SIMD floor, z-chunk, then
# the same for the fused-prolongation sweep; 32 x-pairs):
# build/libmgmc_exps<shape>.so
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
# 27-point z-march variants: slab rows SR x minimum nx (build/libmgmc_expq<SR>x<MIN>.so; MIN above
# every level's nx = the pair / quad passes)
for q in ${Z27S:-}; do
  IFS=x read -r sr mn ex <<< "$q"
  $HIPX -DMGMC_Z27_EXPERIMENT -DMGMC_Z27_SR=$sr -DMGMC_Z27_MIN_NX=$mn ${ex:+-DMGMC_Z27_EXP=$ex} \
    -o ../../build/libmgmc_expq$q.so $SRCS &
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
# k_tail timing builds (MGMC_TAIL_EXP, mgmc_tail.hpp): 1 no noise draws, 2 no colour-pass updates
# (build/libmgmc_expt<N>.so; wrong samples, timing only)
for n in ${TAILEXPS:-}; do
  $HIPX -DMGMC_TAIL_EXP=$n -o ../../build/libmgmc_expt$n.so $SRCS &
done
# coarse SSOR kernel timing build (MGMC_COARSE_EXP=1: no noise draws; build/libmgmc_expc1.so)
for n in ${COARSEEXPS:-}; do
  $HIPX -DMGMC_COARSE_EXP=$n -o ../../build/libmgmc_expc$n.so $SRCS &
done
wait
