"""Same-box A/B of bench.py under environment variants (library path, schedule, ...), interleaved reps.
usage (GPU box): python tools/ab_env.py <tag> "<configs>" name=ENV=VAL[,ENV=VAL] ... [--reps 2]
'prod' (no change) always runs first. Writes gpurun_out/<tag>_<config>_<name>_<rep>.json and prints a table."""
import json
import os
import subprocess
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "gpurun_out")


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--reps")]
    reps = int(next((a.split("=")[1] for a in sys.argv[1:] if a.startswith("--reps=")), 2))
    tag, configs, specs = args[0], args[1].split(), args[2:]
    variants = [("prod", {})]
    for s in specs:
        name, _, env = s.partition("=")
        kv = {}
        for item in env.split(","):
            k, _, v = item.partition("=")
            kv[k] = v.replace("@ROOT", ROOT)
        variants.append((name, kv))
    os.makedirs(OUT, exist_ok=True)
    rows = []
    for rep in range(1, reps + 1):
        for c in configs:
            for name, kv in variants:
                env = dict(os.environ, **kv)
                path = os.path.join(OUT, f"{tag}_{c}_{name}_{rep}.json")
                with open(path, "w") as fh:
                    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", c, "--steps", "60",
                                        "--no-cpu-baseline"], stdout=fh, stderr=subprocess.DEVNULL, env=env,
                                       timeout=300)
                if r.returncode != 0:
                    print(f"STOP {c} {name} rc={r.returncode}")
                    sys.exit(r.returncode)
                d = json.load(open(path))
                k = (d.get("roofline") or {}).get("kernel_ms_mean")
                rows.append((c, name, rep, d["value"], d["ms_per_step"], k, d["qp_iter_mean"], d["qp_iter_max"],
                             d["failed_solves"]))
                print(*rows[-1], flush=True)


if __name__ == "__main__":
    main()
