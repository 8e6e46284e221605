# Shader clock and power sampled by amd-smi while the two-try bench runs (dev tool): is the
# headline regime clock-limited?  Output: gpurun_out/clock_samples.log, gpurun_out/clock_bench.json
set -e
mkdir -p gpurun_out
rm -f gpurun_out/clock_samples.log
STEPS=${STEPS:-200}
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-other-configs --steps $STEPS --warmup 3 > gpurun_out/clock_bench.json 2> gpurun_out/clock_bench.err &
BP=$!
for i in $(seq 1 60); do
  kill -0 $BP 2>/dev/null || break
  echo "T $(date +%s.%N)" >> gpurun_out/clock_samples.log
  timeout -k 5 20 amd-smi metric -g 0 --clock --power >> gpurun_out/clock_samples.log 2>&1 || true
  sleep 0.3
done
wait $BP
python3 - <<'PY'
import re
cur = None; rows = []
for line in open("gpurun_out/clock_samples.log"):
    if line.startswith("T "):
        cur = {"t": float(line.split()[1]), "gfx": []}; rows.append(cur)
    elif "SOCKET_POWER" in line and cur is not None:
        m = re.search(r"(\d+) W", line); cur["w"] = int(m.group(1)) if m else None
    elif re.match(r"\s+CLK: \d+ MHz", line) and cur is not None and len(cur["gfx"]) < 8:
        cur["gfx"].append(int(line.split()[1]))
t0 = rows[0]["t"] if rows else 0
for r in rows:
    g = r["gfx"]
    print("t %6.1f s  power %s W  gfx clock mean %s MHz (min %s max %s)" % (r["t"] - t0, r.get("w"), sum(g) // max(1, len(g)), min(g or [0]), max(g or [0])))
PY
tail -1 gpurun_out/clock_bench.json | cut -c1-200
