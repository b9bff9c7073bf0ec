scripts/gpu_step.sh tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
bash scripts/_ab.sh "$@"
