# Diagnostic library with phase timestamps (SGMM_STAMPS) -> tools/stamps/libsgmm_stamps.so
set -e
D=deep-reinforcement-learning-based-signal-gated-market-making_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 -DSGMM_STAMPS \
  -o tools/stamps/libsgmm_stamps.so $D/sgmm_capi.hip $D/sgmm_rollout.hip $D/sgmm_ga.hip $D/sgmm_bundle.hip $D/sgmm_sgu2.hip
