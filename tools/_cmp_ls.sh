for kv in "$@"; do
  tag=${kv%%=*}; envs=${kv#*=}
  env $envs timeout -k 10 200 python bench.py --model lsgan --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/ls_$tag.log 2>&1 || exit 1
done
