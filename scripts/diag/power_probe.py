"""Socket power and shader clock while the c2 queue kernel runs (diagnostic): for each
diagnostic mode (40 production, 50002 memory-only, 50004 compute-only) a child process
runs scripts/diag/queue_ab.py with many steps while this process samples
`rocm-smi --showpower --showclocks --json` (a sysfs read, no GPU work); prints the
median power / sclk / mclk over the samples taken while the child ran.
usage: python3 scripts/diag/power_probe.py [steps] [mode[:steps[:delay]] ...]
(modes: 40 production, 50002 no arithmetic, 50004 no global memory, 50768 no LDS exchange,
50772 arithmetic only, 50770 global memory only; per-mode steps so each runs ~10 s)
"""
import json
import os
import re
import statistics
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def sample():
    r = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"], capture_output=True, text=True,
                       timeout=20)
    try:
        d = json.loads(r.stdout)
    except ValueError:
        return None
    card = d.get("card0") or next(iter(d.values()), {})
    out = {}
    for k, v in card.items():
        kl = k.lower()
        num = re.search(r"([0-9.]+)", str(v))
        if not num:
            continue
        # rocm-smi reports "<clk> clock speed:" = "(1500Mhz)" and "<clk> clock level:" = "1":
        # only the speed entries are clocks (the level index once overwrote them)
        if "power" in kl and "w" in kl:
            out["power_W"] = float(num.group(1))
        elif kl.startswith("sclk") and "speed" in kl:
            out["sclk_MHz"] = float(num.group(1))
        elif kl.startswith("mclk") and "speed" in kl:
            out["mclk_MHz"] = float(num.group(1))
    return out


def main(steps, modes=("40", "50002", "50004")):
    raw = subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"], capture_output=True, text=True,
                         timeout=20).stdout
    print(json.dumps({"rocm_smi_raw": raw[:1500]}), flush=True)
    idle = [s for s in (sample() for _ in range(3)) if s]
    print(json.dumps({"mode": "idle", "samples": idle}), flush=True)
    for m in modes:
        mode, _, rest = m.partition(":")
        st, _, delay = rest.partition(":")
        env = dict(os.environ, QAB_STEPS=st or str(steps))
        child = subprocess.Popen([sys.executable, os.path.join(HERE, "queue_ab.py"), f"queue,256,3,{delay or 2},{mode}"],
                                 env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        time.sleep(4.0)  # context creation, buffers, warmup
        got = []
        while child.poll() is None:
            s = sample()
            if s:
                got.append(s)
            time.sleep(0.2)
        res = child.stdout.read().strip().splitlines()
        line = next((json.loads(l) for l in reversed(res) if l.startswith("{")), None)
        summ = {k: statistics.median([g[k] for g in got if k in g]) for k in ("power_W", "sclk_MHz", "mclk_MHz")
                if any(k in g for g in got)}
        print(json.dumps({"mode": mode, "delay": int(delay or 2), "samples": len(got), **summ, "run": line}), flush=True)
        if child.returncode:
            print("\n".join(res[-20:]), file=sys.stderr)
            sys.exit(1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000, tuple(sys.argv[2:]) or ("40", "50002", "50004"))
