"""Socket power while a command runs (diagnostic): samples `rocm-smi --showpower --json`
every 0.2 s after a settle delay and prints the command's last JSON line with the median
power.  usage: python3 scripts/diag/power_cmd.py <settle_s> <command...>"""
import json
import statistics
import subprocess
import sys
import time

from power_probe import sample


def main():
    settle = float(sys.argv[1])
    idle = [s["power_W"] for s in (sample() for _ in range(3)) if s and "power_W" in s]
    child = subprocess.Popen(sys.argv[2:], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    time.sleep(settle)
    got = []
    while child.poll() is None:
        s = sample()
        if s and "power_W" in s:
            got.append(s["power_W"])
        time.sleep(0.2)
    lines = [l for l in child.stdout.read().splitlines() if l.startswith("{")]
    out = json.loads(lines[-1]) if lines else {}
    out.update({"cmd": " ".join(sys.argv[2:]), "power_W": statistics.median(got) if got else None,
                "samples": len(got), "idle_W": statistics.median(idle) if idle else None})
    print(json.dumps(out), flush=True)
    sys.exit(child.returncode)


if __name__ == "__main__":
    main()
