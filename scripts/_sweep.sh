# A/B timing sweep of schedule settings within one box: chol_sweep.py settings
timeout -k 10 300 python scripts/chol_sweep.py "$@" > gpurun_out/sweep.log 2>&1 || exit 1
python - <<'PY'
import json
for l in open('gpurun_out/sweep.log'):
    if l.startswith('{'):
        d = json.loads(l)
        print(d['w4_min'], d['w8_min'], d['serial_below'], round(d['ms_median'], 3), round(d['ms_min'], 3), d['mll'])
PY
