# A/B variant of libsgmm.so built with extra -D flags: tools/variants/libsgmm_<name>.so
# (always -DSGMM_EXPERIMENTS: the variant takes its initial launch-plan overrides from
# the SGMM_* environment variables, which the shipped library never reads)
# usage: bash tools/build_variant.sh NAME -DFLAG[=V] ...   (run it with SGMM_LIB=tools/variants/libsgmm_NAME.so)
set -e
name=$1; shift
mkdir -p tools/variants
python deep-reinforcement-learning-based-signal-gated-market-making_amd/build.py \
  --out tools/variants/libsgmm_$name.so -- -DSGMM_EXPERIMENTS "$@"
