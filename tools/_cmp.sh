# A/B of the default library under env settings: bash tools/_cmp.sh "TAG=ENV" ...
for kv in "$@"; do
  tag=${kv%%=*}; envs=${kv#*=}
  env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 > gpurun_out/v_$tag.log 2>&1 || exit 1
done
