set -o pipefail
mkdir -p gpurun_out/small
for O in "" "--opt attn_fuse=1"; do
  TURTLE_BENCH_DUMP=gpurun_out/small/d.tsv timeout -k 10 200 python -u bench.py --res 256 --steps 30 --warmup 5 --no-cpu-baseline --no-psnr $O > gpurun_out/small/l.log 2>&1 || exit 1
  echo "opt[$O]: $(tail -1 gpurun_out/small/l.log | cut -c1-150)"
  python3 tools/launch_report.py gpurun_out/small/d.tsv --steps 5 --top 25 > gpurun_out/small/r$([ -z "$O" ] && echo 0 || echo 1).txt
done
head -30 gpurun_out/small/r0.txt
