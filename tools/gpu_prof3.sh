# round-2 profile refresh: configs 3, 2, 4 (kernel trace, PMC traffic, SQ counters, bench line)
set -o pipefail
for C in 3 2 4; do
  bash tools/r02_profile.sh r02c $C || exit 1
done
