#!/usr/bin/env python3
"""Interleaved A/B of bench.py variants on one box (round 4's single A/B
driver; replaces the per-experiment shell scripts of earlier rounds).

    python tools/ab.py [--reps R] [--timeout S] [--env K=V ...] NAME::ARGS ...

Each variant is `bench.py ARGS --no-cpu --no-traffic` in a child process
(this parent never touches the GPU), run R times round-robin so box drift
hits every variant alike.  Prints one summary line per variant: kernel ms
(mean of the per-run HIP-event averages), roofline frac, ms_per_step, and the
launch (mode / grid / shape).  Full JSON lines go to gpurun_out/ab/<NAME>.jsonl.
A variant that fails stops the whole run (no retries on the GPU).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--timeout", type=int, default=240)
    ap.add_argument("--env", action="append", default=[], help="NAME=K=V: extra env for one variant")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out", "ab")
    os.makedirs(out, exist_ok=True)
    vs = []
    for v in a.variants:
        name, _, args = v.partition("::")
        vs.append((name, args.split()))
    extra = {}
    for e in a.env:
        name, kv = e.split("=", 1)
        k, val = kv.split("=", 1)
        extra.setdefault(name, {})[k] = val
    res = {n: [] for n, _ in vs}
    for rep in range(a.reps):
        for name, args in vs:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args, "--no-cpu", "--no-traffic"]
            env = dict(os.environ, **extra.get(name, {}))
            p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout)
            with open(os.path.join(out, name + ".err"), "a") as f:
                f.write(p.stderr)
            if p.returncode != 0:
                print(f"{name}: exit {p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(p.returncode)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
            with open(os.path.join(out, name + ".jsonl"), "a") as f:
                f.write(line + "\n")
            j = json.loads(line)
            res[name].append(j)
            r = j.get("roofline") or {}
            print(f"  rep {rep} {name:24s} kernel {r.get('kernel_ms_avg', j.get('kernel_ms_avg'))} "
                  f"frac {r.get('frac', j.get('frac_of_8TBs'))} step {j.get('ms_per_step')}", flush=True)
    print("== summary")
    for name, _ in vs:
        js = res[name]
        if not js:
            continue
        ks = [(j.get("roofline") or {}).get("kernel_ms_avg", j.get("kernel_ms_avg")) for j in js]
        fr = [(j.get("roofline") or {}).get("frac", j.get("frac_of_8TBs")) for j in js]
        st = [j.get("ms_per_step") for j in js]
        launch = ((js[0].get("config") or {}).get("launch")) if isinstance(js[0].get("config"), dict) else None
        print(f"{name:24s} kernel {sum(ks) / len(ks):.5f} ms (min {min(ks):.5f}) frac {sum(fr) / len(fr):.4f} "
              f"(max {max(fr):.4f}) step {sum(st) / len(st):.4f} {launch}", flush=True)


if __name__ == "__main__":
    main()
