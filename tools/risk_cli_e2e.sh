#!/bin/bash
# demo.py-equivalent CLI end to end on a synthetic barra_data_csi.csv: wall time of each phase.
# usage: tools/risk_cli_e2e.sh DATES STOCKS  (writes under gpurun_out/cli_e2e)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=${1:-1250}; N=${2:-300}
O=${TMPDIR:-/tmp}/cli_e2e_${D}x${N}; rm -rf $O; mkdir -p $O  # big CSVs: keep out of gpurun_out
t0=$(date +%s.%N)
timeout -k 10 300 python -m llm_driven_multi_factor_model_amd.cli synth --out $O/data --dates $D --stocks $N --industries 31 > $O/synth.log 2>&1 || exit 1
t1=$(date +%s.%N)
timeout -k 10 300 python -m llm_driven_multi_factor_model_amd.cli risk --data $O/data/barra_data_csi.csv --industry $O/data/industry_info.csv --out $O/res > $O/risk.log 2>&1 || exit 1
t2=$(date +%s.%N)
ls -la $O/data $O/res >&2
python3 - "$t0" "$t1" "$t2" "$O" <<'PY'
import sys, json
t0, t1, t2, o = float(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3]), sys.argv[4]
log = open(f"{o}/risk.log").read().splitlines()
print(json.dumps({"synth_s": round(t1 - t0, 2), "risk_cli_s": round(t2 - t1, 2),
                  "log": [l.split(": ", 1)[-1][:200] for l in log if "loaded" in l or "stage ms" in l or "wrote" in l]}))
PY
