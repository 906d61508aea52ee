#!/bin/bash
# Compressed TeraSort MOFs in HBM through the C ABI (16 tasks decode every block on the device straight
# from the descriptors), Snappy and LZO1X: device decodes taking turns (mapred.uda.gpu.decode.slots =
# 1, default; 2) vs all at once (0).
set -o pipefail
mkdir -p gpurun_out
for c in ${CODECS:-snappy lzo}; do
  for sl in ${SLOTS:-1 0 2}; do
    log=gpurun_out/r3_bench_api_${c}_41GB_slots$sl.log
    UDA_API_CONF="mapred.uda.gpu.decode.slots=$sl" timeout -k 10 600 python -u bench.py --api --api-codec $c \
      --rows-per-gpu 400000000 --steps 3 --warmup 1 > $log 2>&1 || { tail -30 $log; exit 1; }
    echo "$c slots=$sl $(grep -o '"value": [0-9.]*\|"validated": [a-z]*\|"compressed_gb": [0-9.]*' $log | tr '\n' ' ') $(grep -o '"gpu_decode_ms": [0-9.]*\|"total_ms": [0-9.]*\|"gpu_sink_ms": [0-9.]*' $log | tr '\n' ' ')"
  done
done
