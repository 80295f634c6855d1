#!/usr/bin/env python3
"""Run tools/dz_probe.py once per timing variant (child processes; this one never touches
the GPU) and print its JSON lines: per-well / joint chains x natural / transformed space x
NGRTD_DZ_DIAG variants (0 full, 16 no partner loads, 1 proposal = state, 8 no staging,
4 no commit).

    python tools/dz_variants.py [--diags 0,16,1,8,4] [--models exponential]
                                [--envs none,NGRTD_DZ_STATE_GLOBAL=1+NGRTD_DZ_PROP_GLOBAL=1]
--envs: extra environment per variant ("none"; K=V pairs joined by "+")."""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--diags", default="0,16,1,8,4")
    ap.add_argument("--models", default="exponential")
    ap.add_argument("--pw", default="1,0")
    ap.add_argument("--jac", default="1,0")
    ap.add_argument("--envs", default="none")
    a = ap.parse_args()
    for model, ev in [(m, e) for m in a.models.split(",") for e in a.envs.split(",")]:
        for pw in a.pw.split(","):
            for jac in a.jac.split(","):
                for dg in a.diags.split(","):
                    env = dict(os.environ, NGRTD_DZ_DIAG=dg, DZ_PW=pw)
                    extra = dict(kv.split("=", 1) for kv in ev.split("+")) if ev != "none" else {}
                    env.update(extra)
                    if model != "exponential":
                        env["DZ_MODEL"] = model
                    if jac == "1":
                        env["DZ_JAC"] = "1"
                    else:
                        env.pop("DZ_JAC", None)
                    r = subprocess.run([sys.executable, os.path.join(HERE, "dz_probe.py")], env=env, timeout=300,
                                       capture_output=True, text=True)
                    if r.returncode:
                        print('{"error": %r}' % r.stderr[-500:], flush=True)
                        sys.exit(r.returncode)
                    line = json.loads(r.stdout.strip().splitlines()[-1])
                    line["env"] = extra
                    print(json.dumps(line), flush=True)
