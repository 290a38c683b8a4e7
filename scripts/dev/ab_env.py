"""A/B of library knobs set through the environment: runs `bench.py ARGS` once per form and
repetition, alternating the forms, and prints value and per-stage launch times per run.

    python scripts/dev/ab_env.py REPS "label:VAR=V,VAR2=V" ["label2:..."] -- bench args..."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]


def main():
    reps = int(sys.argv[1])
    cut = sys.argv.index("--")
    forms = sys.argv[2:cut]
    args = sys.argv[cut + 1:]
    for r in range(reps):
        for f in forms:
            label, _, envs = f.partition(":")
            env = dict(os.environ)
            for kv in filter(None, envs.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(label, "rc", p.returncode, p.stderr[-2000:], flush=True)
                sys.exit(p.returncode)
            line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
            st = (line.get("latency") or {}).get("stages", {})
            print(json.dumps({"rep": r, "form": label, "value": line["value"],
                              "stages_us": {k: round(v["ms_per_launch"] * 1000, 2)
                                            for k, v in st.items()}}), flush=True)


if __name__ == "__main__":
    main()
