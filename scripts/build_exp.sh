# Tuning builds of the library into build/ (never the product; select one with
# MGMC_LIBRARY=build/libmgmc_<name>.so).  The product sources carry no override switches: every
# launch-shape constant lives in multigridmc_amd/csrc/mgmc_tuning.hpp (bitwise-neutral: tile shapes,
# chunk depths, thread counts, launch thresholds).  A variant is a copy of the sources with some of
# those constants edited:
#   VARIANTS="ty16=ZS_TY:16 nt256=QUADS_NT:256,QUADS_NT3:256" bash scripts/build_exp.sh
# builds build/libmgmc_ty16.so and build/libmgmc_nt256.so.  CXXDEFS="-DMGMC_TAIL_PROF" adds
# compile definitions to every variant (the k_tail phase stamps of scripts/tail_prof.py).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/build"
HIPX="/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -w --offload-arch=gfx950 -shared ${CXXDEFS:-}"
LIBS="-L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib"
pids=""
for v in ${VARIANTS:-}; do
  name=${v%%=*}; edits=${v#*=}
  rm -f "$ROOT/build/libmgmc_$name.so"  # a failed compile must not leave an older build to be A/B'd
  src="$ROOT/build/exp_$name"
  rm -rf "$src" && mkdir -p "$src/multigridmc_amd" "$src/include"
  cp -r "$ROOT/multigridmc_amd/csrc" "$src/multigridmc_amd/"
  cp "$ROOT"/include/*.h "$src/include/"
  tun="$src/multigridmc_amd/csrc/mgmc_tuning.hpp"
  for e in ${edits//,/ }; do
    key=${e%%:*}; val=${e#*:}
    [ "$key" = "-" ] && continue
    grep -q "constexpr int $key = " "$tun" || { echo "build_exp: no constant $key in mgmc_tuning.hpp" >&2; exit 2; }
    sed -i "s/constexpr int $key = [^;]*;/constexpr int $key = $val;/" "$tun"
  done
  (cd "$src/multigridmc_amd/csrc" && $HIPX -o "$ROOT/build/libmgmc_$name.so" *.hip *.cpp $LIBS) &
  pids="$pids $!"
done
for p in $pids; do wait "$p" || { echo "build_exp: a variant failed to compile" >&2; exit 1; }; done
