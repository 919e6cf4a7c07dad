#!/usr/bin/env bash
# Onebox start-up (the reference's DeploymentLocal/finalrun.sh role): start the control plane + web console, load the
# sample flows, optionally start them.  Everything stays on this machine; jobs run one process per GPU.
set -euo pipefail
ROOT=${DXA_ROOT:-$PWD/.dxa}
PORT=${DXA_PORT:-5000}
HERE=$(cd "$(dirname "$0")" && pwd)
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DXA_SECRETS_DIR=${DXA_SECRETS_DIR:-$ROOT/secrets}
mkdir -p "$ROOT"
python -m dxa.service.app --host 0.0.0.0 --port "$PORT" --root "$ROOT" &
PID=$!
trap 'kill $PID' EXIT
for i in $(seq 1 60); do
  curl -sf "http://127.0.0.1:$PORT/api/health" >/dev/null && break
  sleep 1
done
for f in "$HERE"/samples/*.json; do
  [ -e "$f" ] || continue
  curl -sf -X POST -H 'Content-Type: application/json' --data @"$f" "http://127.0.0.1:$PORT/api/flow/save" >/dev/null
  echo "loaded sample flow $(basename "$f")"
done
if [ "${DXA_START_SAMPLES:-0}" = "1" ]; then
  for f in "$HERE"/samples/*.json; do
    name=$(python -c "import json,sys; print(json.load(open(sys.argv[1]))['name'])" "$f")
    curl -sf -X POST -H 'Content-Type: application/json' --data "\"$name\"" "http://127.0.0.1:$PORT/api/flow/startjobs"
  done
fi
wait $PID
