# Diagnostic library with phase timestamps (SGMM_STAMPS) -> tools/stamps/libsgmm_stamps.so
set -e
mkdir -p tools/stamps
python deep-reinforcement-learning-based-signal-gated-market-making_amd/build.py \
  --out tools/stamps/libsgmm_stamps.so -- -DSGMM_STAMPS -DSGMM_EXPERIMENTS "$@"
