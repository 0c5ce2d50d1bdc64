set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PROF_STEPS=7 ROUND=r05b bash tools/gpu_round.sh prof stages || exit $?
