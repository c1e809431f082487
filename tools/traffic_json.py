"""profiles/traffic_<key>_b<B>.json (bench.py's roofline.traffic and .valu) from a
tools/summarize_profile.py summary:
    python tools/traffic_json.py profiles/<tag>/summary.json <key> <T> <B> <alg bytes per env-step>
<key> is bench.py's traffic key: <config>_rollout<T> for a T-step rollout launch, <config>_ring32
for the per-step launch into a 32-slot ring (T = 1)."""
import json
import sys


def main(summary, key, T, B, alg_per_env_step):
    s = json.load(open(summary))
    T, B, alg = int(T), int(B), float(alg_per_env_step)
    hbm = s["hbm_bytes_per_launch"]
    alg_launch = alg * B * T
    out = {"config": "%s (%d steps per launch), B=%d" % (key, T, B), "kernel": s["trace"]["name"],
           "avg_ns": s["trace"]["avg_ns"], "hbm_bytes_per_launch": hbm, "alg_bytes_per_launch": alg_launch,
           "traffic_over_alg": hbm["total_corrected"] / alg_launch, "valu": s.get("valu"),
           "source": summary.rsplit("/", 1)[0]}
    path = "profiles/traffic_%s_b%d.json" % (key, B)
    json.dump(out, open(path, "w"), indent=1)
    print(path, json.dumps({k: out[k] for k in ("avg_ns", "traffic_over_alg")}))


if __name__ == "__main__":
    main(*sys.argv[1:])
