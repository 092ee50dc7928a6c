# Build a library from a git revision's csrc into tools/diag/libsgmm_<tag>.so (A/B timing).
# Usage: bash tools/ab_lib.sh <rev> <tag>
set -e
R=${1:-HEAD}; T=${2:-head}
D=/tmp/ab_$T; rm -rf $D; mkdir -p $D/csrc $D/include
P=deep-reinforcement-learning-based-signal-gated-market-making_amd/csrc
git archive $R $P include | tar -x -C $D
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 \
  -o tools/diag/libsgmm_$T.so $D/$P/sgmm_capi.hip $D/$P/sgmm_rollout.hip $D/$P/sgmm_ga.hip $D/$P/sgmm_bundle.hip $D/$P/sgmm_sgu2.hip
