set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl
AB_REPS=3 timeout -k 10 900 bash tools/x3_ab.sh f32 ${VARIANTS} > /dev/null 2>&1
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l); d[j["lib"]].append((j["agg_rows"], j["agg_color"], j["frame"]))
for k, v in d.items():
    print(k, "rows", [round(x[0], 2) for x in v], "color", [round(x[1], 3) for x in v], "frame", [round(x[2], 2) for x in v])
PY
