"""profiles/rNN/sim_ranks.json from tools/sim_ranks.sh output: every rank's
shard of the N-rank plan run alone on one GPU; the slowest rank bounds the
N-GPU step (collectives excluded).
usage: python tools/sim_summary.py <sim dir> <bench_full.json> <out.json>"""
import glob
import json
import re
import sys

sim, bench, out = sys.argv[1:4]
last = lambda f: json.loads(open(f).read().strip().splitlines()[-1])  # noqa: E731
n1 = last(bench)["ms_per_step"]
plans = {}
for f in sorted(glob.glob(f"{sim}/*_n*_r*.json")):
    m = re.search(r"_n(\d+)_r(\d+)\.json$", f)
    j = last(f)
    plans.setdefault(m.group(1), {"ranks": []})["ranks"].append(
        {"rank": int(m.group(2)), "shard_bp": j["shard_bp"], "ms_per_step": j["ms_per_step"],
         "k1a_ms": j["k1a_ms"], "warmup_timings_ms": j["warmup_timings_ms"]})
for p in plans.values():
    p["ranks"].sort(key=lambda r: r["rank"])
    p["max_ms_per_step"] = max(r["ms_per_step"] for r in p["ranks"])
    p["speedup_vs_n1"] = round(n1 / p["max_ms_per_step"], 3)
json.dump({"what": "compute side of an N-GPU strong-scaling run on a one-GPU box: every rank's shard of "
                   "the N-rank LPT plan run alone (bench.py with UNIPEAK_SIM_WORLD/UNIPEAK_SIM_RANK, "
                   "tools/sim_ranks.sh); the slowest rank bounds the N-GPU step (collectives excluded)",
           "n1_ms_per_step": n1, "plans": dict(sorted(plans.items(), key=lambda kv: int(kv[0])))},
          open(out, "w"), indent=1)
print({k: (v["max_ms_per_step"], v["speedup_vs_n1"]) for k, v in plans.items()})
