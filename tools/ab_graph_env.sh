set -o pipefail
mkdir -p gpurun_out/r6e
for rep in 1 2 3; do
  for cfg in base pc0 pc1 dk0 dk1; do
    case $cfg in
      base) E="" ;;
      pc0) E="DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" ;;
      pc1) E="DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" ;;
      dk0) E="HIP_FORCE_DEV_KERNARG=0" ;;
      dk1) E="HIP_FORCE_DEV_KERNARG=1" ;;
    esac
    env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-convergence --no-anchor --no-fp32 --trace-rounds 0 > gpurun_out/r6e/$cfg.$rep.log 2>&1 || exit 1
    echo "$cfg $rep $(grep -o '"us_per_round": [0-9.]*' gpurun_out/r6e/$cfg.$rep.log | head -1)" | tee -a gpurun_out/r6e/summary.txt
  done
done
