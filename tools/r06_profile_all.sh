# Round 6 evidence for every BASELINE shape and per-rank shard (tools/r06_profile.sh each)
set -o pipefail
for spec in "c3:--config 3" "c2:--config 2" "c6:--config 6" "c4:--config 4" "c4s4:--config 4 --shard-of 4" \
            "c5:--config 5" "c5s2:--config 5 --shard-of 2" "c5s4:--config 5 --shard-of 4" \
            "c5s8:--config 5 --shard-of 8" "c5s16:--config 5 --shard-of 16"; do
  name=${spec%%:*}; args=${spec#*:}
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then continue; fi
  echo "== $name"
  bash tools/r06_profile.sh r06prof/$name $args || exit 1
done
