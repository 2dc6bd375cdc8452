#!/usr/bin/env bash
# One-node MI355X bring-up + the reference's three jobs (mirrors a3-mega/gke-ray-cluster-setup.sh:
# exports -> cluster -> job submissions), with the GKE/KubeRay/GCS-FUSE steps replaced by the
# node-local grt head.  Usage: deploy/mi355x/cluster-setup.sh [--cpu-smoke]
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
GRT="$ROOT/bin/grt"

export CLUSTER_NAME="${CLUSTER_NAME:-grt-mi355x}"
export NUM_NODES=1
export NUM_GPUS_PER_NODE="${NUM_GPUS_PER_NODE:-8}"
export STORAGE_PATH="${STORAGE_PATH:-/tmp/grt_storage}"
export DASHBOARD_PORT="${DASHBOARD_PORT:-8265}"
SMOKE=0
if [[ "${1:-}" == "--cpu-smoke" ]]; then SMOKE=1; export NUM_GPUS_PER_NODE=0; fi

"$GRT" cluster up -f "$ROOT/deploy/mi355x/cluster.yaml"
trap '"$GRT" cluster down >/dev/null 2>&1 || true' EXIT
ADDR="http://127.0.0.1:${DASHBOARD_PORT}"

ENV_JSON=$(printf '{"env_vars": {"NUM_NODES": "%s", "NUM_GPUS_PER_NODE": "%s", "GRT_PVC": "%s"}}' \
  "$NUM_NODES" "$NUM_GPUS_PER_NODE" "$STORAGE_PATH")

# 1) data prep (Ray Core task)          ~ ray-jobs/prepare_wikitext2_ray_job.py
"$GRT" job submit --address "$ADDR" --working-dir "$ROOT" --runtime-env-json "$ENV_JSON" -- \
  python jobs/prepare_wikitext2_ray_job.py --scale "${DATA_SCALE:-1.0}"

if [[ $SMOKE == 1 ]]; then
  # 2) BasicLLM DDP (config #1: 2 CPU workers, gloo)
  "$GRT" job submit --address "$ADDR" --working-dir "$ROOT" --runtime-env-json "$ENV_JSON" -- \
    python jobs/pytorch_llm_ray.py --cpu --workers 2 --preset tiny --max-windows 512
  exit 0
fi
# 2) BasicLLM DDP on all GPUs            ~ ray-jobs/pytorch_llm_ray.py
"$GRT" job submit --address "$ADDR" --working-dir "$ROOT" --runtime-env-json "$ENV_JSON" -- \
  python jobs/pytorch_llm_ray.py --workers "$NUM_GPUS_PER_NODE"
# 3) Llama SFT (QLoRA or full FT per fine_tune_config.json)  ~ ray-jobs/fine_tune_llama_ray.py
"$GRT" job submit --address "$ADDR" --working-dir "$ROOT" --runtime-env-json "$ENV_JSON" -- \
  python jobs/fine_tune_llama_ray.py
