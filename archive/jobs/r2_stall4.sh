source tools/gpu_job.sh
export DDL_HOST_LOG=1 DDL_STAGER_LOG=1
AMD_LOG_LEVEL=4 run 120 s_log python bench.py --gpus 1 --steps 12 --warmup 5 --order window --idle-steps 0 --json-out gpurun_out/s_log.json
python - <<'PY'
import re
lines = open("gpurun_out/s_log.log", errors="replace").read().splitlines()
out = []
start = None
for i, l in enumerate(lines):
    if "hipMemcpyAsync (" in l:
        start = i
    m = re.search(r"hipMemcpyAsync: Returned .*duration: (\d+) us", l)
    if m and start is not None:
        if int(m.group(1)) > 1000:
            out.append("=" * 40 + f" slow {m.group(1)} us")
            out += lines[start:i + 1][:400]
        start = None
open("gpurun_out/s_log_slow.txt", "w").write("\n".join(out[:3000]) + "\n")
PY
rm -f gpurun_out/s_log.log
