# A/B variant of libsgmm.so built with extra -D flags: tools/variants/libsgmm_<name>.so
# usage: bash tools/build_variant.sh NAME -DFLAG[=V] ...   (run it with SGMM_LIB=tools/variants/libsgmm_NAME.so)
set -e
name=$1; shift
D=deep-reinforcement-learning-based-signal-gated-market-making_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 "$@" \
  -o tools/variants/libsgmm_$name.so $D/sgmm_capi.hip $D/sgmm_rollout.hip $D/sgmm_ga.hip $D/sgmm_bundle.hip $D/sgmm_sgu2.hip
