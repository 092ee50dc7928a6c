# config-5 evidence: rocprofv3 kernel stats, PMC traffic, SQ counters, bench line
set -o pipefail
bash tools/r02_profile.sh r02h 5
