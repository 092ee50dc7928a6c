# rocprofv3 kernel trace of a config-3 bench run (graph replays + eager profile steps)
set -o pipefail
D=gpurun_out/kt3; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- python bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --profile-steps 5 > $D/b.json 2> $D/kt.err || { echo KT_FAIL; tail $D/kt.err; exit 1; }
cp $(find $D/kt -name "*kernel_stats.csv" | head -1) $D/kernel_stats.csv
cut -d, -f1-8 $D/kernel_stats.csv | head -12
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/kt3/kt/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0][:60]
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    v2 = sorted(v)
    print(f"{n:60s} n={len(v):4d} med {v2[len(v2)//2]:8.1f} min {v2[0]:8.1f} max {v2[-1]:8.1f} us")
PY
