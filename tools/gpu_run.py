#!/usr/bin/env python3
"""One parametrized GPU-box runner (replaces the per-experiment gpurun shell recipes).

    gpurun --timeout 1100 -- 'python3 tools/gpu_run.py --tag r4 pytest smoke bench api41'
    gpurun -- 'python3 tools/gpu_run.py --tag ab --cmd "sec48x=400=python -u bench.py --api ..." sec48'

Every step runs under its own time limit in its own process group, stdout goes to
gpurun_out/<tag>_<name>.log and stderr to .err. The runner prints one summary line per step (the
JSON line a bench prints: value, validated, plus --keys) and stops at the first failing step: after
a fault, an abort, a crash or a time limit nothing else may use the GPU in that call.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PY = "python3 -u"

# name -> (seconds, command). Commands run from the repo root through bash.
RECIPES: dict[str, tuple[int, str]] = {
    "pytest": (900, f"{PY} -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread"),
    "smoke": (300, f"{PY} -c 'import __graft_entry__ as g; g.smoke()'"),
    "bench": (400, f"{PY} bench.py --steps 3 --warmup 1"),
    "device_only": (300, f"{PY} bench.py --device-only --steps 3 --warmup 1"),
    "api41": (400, f"{PY} bench.py --api --rows-per-gpu 400000000 --steps 3 --warmup 1"),
    "api130": (500, f"{PY} bench.py --api --steps 3 --warmup 1"),
    "api_files41": (600, f"{PY} bench.py --api --mof-dir /tmp/uda_mofs --rows-per-gpu 400000000 --steps 2 --warmup 0"),
    "api2_one_gpu": (500, f"{PY} bench.py --api --gpus 2 --one-gpu --rows-per-gpu 400000000 --steps 3 --warmup 1"),
    "api4_one_gpu": (500, f"{PY} bench.py --api --gpus 4 --one-gpu --rows-per-gpu 200000000 --steps 3 --warmup 1"),
    "sec48": (400, f"{PY} bench.py --api --workload secondary --rows-per-gpu 470000000 --steps 3 --warmup 1"),
    "sec100": (600, f"{PY} bench.py --api --workload secondary --rows-per-gpu 970000000 --steps 2 --warmup 1"),
    "sec2_one_gpu": (600, f"{PY} bench.py --api --workload secondary --gpus 2 --one-gpu --rows-per-gpu 235000000 --steps 3 --warmup 1"),
    "snappy41": (400, f"{PY} bench.py --api --api-codec snappy --rows-per-gpu 400000000 --steps 3 --warmup 1"),
    "snappy130": (600, f"{PY} bench.py --api --api-codec snappy --steps 2 --warmup 1"),
    "snappy130x5": (600, f"{PY} bench.py --api --api-codec snappy --steps 5 --warmup 1 --verbose"),
    "lzo130x5": (600, f"{PY} bench.py --api --api-codec lzo --steps 5 --warmup 1 --verbose"),
    "lzo41": (400, f"{PY} bench.py --api --api-codec lzo --rows-per-gpu 400000000 --steps 3 --warmup 1"),
    "ipc2": (400, f"{PY} bench.py --gpus 2 --one-gpu --exchange ipc --rows-per-gpu 300000000 --steps 3 --warmup 1"),
    "ipc4": (400, f"{PY} bench.py --gpus 4 --one-gpu --exchange ipc --rows-per-gpu 150000000 --steps 3 --warmup 1"),
    "ipc8": (600, f"{PY} bench.py --gpus 8 --one-gpu --exchange ipc --rows-per-gpu 240000000 --steps 2 --warmup 1"),
    "ipc4_host": (600, f"{PY} bench.py --gpus 4 --one-gpu --exchange ipc --store host --rows-per-gpu 100000000 --steps 2 --warmup 1"),
    "node": (600, f"{PY} bench.py --api --node --no-node-service --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "node130": (700, f"{PY} bench.py --api --node --no-node-service --reducers 15 --steps 2 --warmup 1"),
    "node_gap": (600, f"{PY} bench.py --api --node --reducers 15 --node-gap 1 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41": (900, f"{PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles62": (1000, f"{PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 600000000 --steps 2 --warmup 1"),
    "hybrid40": (900, f"{PY} benchmarks/run_configs.py hybrid_budget --gb 40 --maps 64 --budget-gb 10 --merge-gb 8"),
    "budget_capi": (600, f"UDA_API_CONF=mapred.uda.gpu.hbm.budget=60000000000,mapred.uda.gpu.merge.bytes=1000000000 "
                         f"{PY} bench.py --api --api-host-mofs --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "apihost2": (600, f"{PY} bench.py --api --api-host-mofs --gpus 2 --one-gpu --rows-per-gpu 200000000 --steps 2 --warmup 1"),
    "coldnode5": (500, f"{PY} tools/cold_task_bench.py --node --repeat 5"),
    "coldnode5_j2c": (500, f"UDA_J2C_THREADS=1 {PY} tools/cold_task_bench.py --node --repeat 5"),
    "coldnode5_inline": (500, f"UDA_J2C_THREADS=0 {PY} tools/cold_task_bench.py --node --repeat 5"),
    "coldnode5_c8": (500, f"{PY} tools/cold_task_bench.py --node --repeat 5 --conf mapred.uda.tcp.connections=8"),
    "hybrid41api": (600, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000,mapred.uda.gpu.merge.bytes=8000000000 "
                         f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 1 --warmup 0"),
    "ipc4_host_nospread": (600, f"UDA_SDMA_H2D_SPREAD=0 {PY} bench.py --gpus 4 --one-gpu --exchange ipc --store host "
                                f"--rows-per-gpu 100000000 --steps 2 --warmup 1"),
    "hostmem": (60, "cat /proc/meminfo | head -5; cat /sys/fs/cgroup/memory.max 2>/dev/null; "
                    "cat /sys/fs/cgroup/memory/memory.limit_in_bytes 2>/dev/null; nproc; "
                    "cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/sys/kernel/yama/ptrace_scope 2>/dev/null; true"),
    "aio20": (300, f"{PY} benchmarks/run_configs.py aio --gb 20 --dir /tmp"),
    "hybrid41b": (600, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000 "
                       f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 1 --warmup 0"),
    "sec100_j2c": (600, f"UDA_J2C_THREADS=1 {PY} bench.py --api --workload secondary --rows-per-gpu 970000000 --steps 2 --warmup 1"),
    "api130_j2c": (500, f"UDA_J2C_THREADS=1 {PY} bench.py --api --steps 3 --warmup 1"),
    "bench_j2c": (400, f"UDA_J2C_THREADS=1 {PY} bench.py --steps 3 --warmup 1"),
    "counters": (90, "timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/counters_avail.txt 2>&1; true"),
    "lzo130_s2": (600, f"UDA_API_CONF=mapred.uda.gpu.decode.slots=2 {PY} bench.py --api --api-codec lzo --steps 5 --warmup 1"),
    "snappy130_s2": (600, f"UDA_API_CONF=mapred.uda.gpu.decode.slots=2 {PY} bench.py --api --api-codec snappy --steps 5 --warmup 1"),
    "apihost2_c8": (600, f"UDA_API_CONF=mapred.uda.tcp.connections=8 {PY} bench.py --api --api-host-mofs --gpus 2 --one-gpu "
                         f"--rows-per-gpu 200000000 --steps 2 --warmup 1"),
    "coldfiles5": (500, f"{PY} tools/cold_task_bench.py --files --repeat 5"),
    "lzo130_s3": (600, f"UDA_API_CONF=mapred.uda.gpu.decode.stream.slots=3 {PY} bench.py --api --api-codec lzo --steps 5 --warmup 1"),
    "lzo130_s4": (600, f"UDA_API_CONF=mapred.uda.gpu.decode.stream.slots=4 {PY} bench.py --api --api-codec lzo --steps 5 --warmup 1"),
    "sec100_inline": (600, f"UDA_J2C_THREADS=0 {PY} bench.py --api --workload secondary --rows-per-gpu 970000000 --steps 2 --warmup 1"),
    "api130_inline": (500, f"UDA_J2C_THREADS=0 {PY} bench.py --api --steps 3 --warmup 1"),
    "aio60": (300, f"{PY} benchmarks/run_configs.py aio --gb 60 --dir /tmp"),
    "coldfiles6": (500, f"{PY} tools/cold_task_bench.py --files --repeat 6"),
    "apihost2_g4": (600, f"{PY} bench.py --api --api-host-mofs --gpus 2 --one-gpu --rows-per-gpu 200000000 --steps 2 --warmup 1 "
                         f"--api-gpu-slots 4"),
    "apihost2_g3": (600, f"{PY} bench.py --api --api-host-mofs --gpus 2 --one-gpu --rows-per-gpu 200000000 --steps 2 --warmup 1 "
                         f"--api-gpu-slots 3"),
    "apihost2_41": (600, f"{PY} bench.py --api --api-host-mofs --gpus 2 --one-gpu --rows-per-gpu 400000000 --steps 3 --warmup 1"),
    "apihost2_s5": (600, f"{PY} bench.py --api --api-host-mofs --gpus 2 --one-gpu --rows-per-gpu 200000000 --steps 5 --warmup 1"),
    "coldfiles6_nopin": (500, f"UDA_J2C_PIN=none {PY} tools/cold_task_bench.py --files --repeat 6"),
    "coldnode5_nopin": (500, f"UDA_J2C_PIN=none {PY} tools/cold_task_bench.py --node --repeat 5"),
    "kwtests": (300, f"{PY} -m pytest tests/test_gpu_terasort.py -m gpu -x -v --timeout 170 --timeout-method thread -k kway"),
    "do_staged": (300, f"UDA_KWAY_STAGED=1 {PY} bench.py --device-only --steps 3 --warmup 1"),
    "do_staged512": (300, f"UDA_KWAY_STAGED=1 UDA_KWAY_CAP=512 {PY} bench.py --device-only --steps 3 --warmup 1"),
    "do_cap1024": (300, f"UDA_KWAY_CAP=1024 {PY} bench.py --device-only --steps 3 --warmup 1"),
    "nodefiles41_c32": (900, f"UDA_STORE_CHUNKS=32 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_4mb": (900, f"UDA_STORE_CHUNKS=64 UDA_STORE_CHUNK_MB=4 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_t4": (900, f"UDA_STORE_AIO_THREADS=4 UDA_STORE_CHUNKS=32 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_blit": (900, f"UDA_STORE_H2D=blit {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_r1": (900, f"UDA_STORE_READ_MB=1 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_r2": (900, f"UDA_STORE_READ_MB=2 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_r4": (900, f"UDA_STORE_READ_MB=4 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_o4": (900, f"UDA_STORE_OPENERS=4 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles41_64mb": (900, f"UDA_STORE_CHUNKS=8 UDA_STORE_CHUNK_MB=64 {PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "diskfree": (60, "df -h /tmp /dev/shm . 2>&1; true"),
    "nodefiles130": (1100, f"{PY} bench.py --api --node --mof-dir /tmp --reducers 15 --steps 2 --warmup 1"),
    "host198": (900, f"{PY} bench.py --store host --rows-per-gpu 1900000000 --steps 2 --warmup 1"),
    "node1": (300, f"{PY} bench.py --api --node --reducers 1 --node-slots 1 --rows-per-gpu 20000000 --maps-per-gpu 32 --steps 3 --warmup 1"),
    "cold": (400, f"{PY} tools/cold_task_bench.py --repeat 2"),
    "coldnode": (400, f"{PY} tools/cold_task_bench.py --node --repeat 3"),
    "nodesvc": (400, f"{PY} bench.py --api --node --node-service --reducers 15 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodesvc130": (500, f"{PY} bench.py --api --node --node-service --reducers 15 --steps 2 --warmup 1"),
    "netmerger": (400, f"{PY} benchmarks/run_configs.py netmerger --gb 2 --maps 64 --reducers 1"),
    "prof_bench": (500, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- "
                        "python3 bench.py --steps 3 --warmup 1"),
    "prof_lzo41": (500, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lzo41 -o run -- "
                        "python3 bench.py --api --api-codec lzo --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "pmc_lzo41": (300, "timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY "
                       "SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_lzo41 -o run -- "
                       "python3 bench.py --api --api-codec lzo --rows-per-gpu 100000000 --steps 1 --warmup 0"),
    # round 6
    "pd_tests": (400, f"{PY} -m pytest tests/test_gpu_generic.py -m gpu -x -v --timeout 170 --timeout-method thread "
                      f"-k 'progressive_direct or hybrid_lpq_rpq or hybrid_checkpoint'"),
    "hybrid41b_s2": (700, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000 "
                          f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "hybrid41b_noprog": (700, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000,mapred.uda.gpu.hybrid.progressive=0 "
                              f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "nodefiles62_store20": (1100, f"{PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 600000000 "
                                  f"--provider-hbm-gb 20 --steps 3 --warmup 1"),
    "decode_tests": (300, f"{PY} -m pytest tests/test_gpu_decode.py -m gpu -x -v --timeout 170 --timeout-method thread"),
    "lzo130x5_wave": (600, f"UDA_LZO_LANE=0 {PY} bench.py --api --api-codec lzo --steps 5 --warmup 1 --verbose"),
    "pmc_lzo41_wave": (300, "UDA_LZO_LANE=0 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS "
                            "SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv "
                            "-d gpurun_out/pmc_lzo41_wave -o run -- python3 bench.py --api --api-codec lzo --rows-per-gpu 100000000 "
                            "--steps 1 --warmup 0"),
    "prof_lzo41_lane": (500, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lzo41_lane -o run -- "
                             "python3 bench.py --api --api-codec lzo --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "prof_lzo41_wave": (500, "UDA_LZO_LANE=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lzo41_wave "
                             "-o run -- python3 bench.py --api --api-codec lzo --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "hybrid41b_t4": (700, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000,mapred.uda.gpu.hybrid.progressive.threads=4 "
                          f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "hybrid41b_p16": (700, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000,mapred.uda.gpu.hybrid.progressive.phases=16 "
                           f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 2 --warmup 1"),
    "lzo130x5_lds": (600, f"UDA_DECODE_WINDOW=lds {PY} bench.py --api --api-codec lzo --steps 5 --warmup 1 --verbose"),
    "snappy130x5_r6": (600, f"{PY} bench.py --api --api-codec snappy --steps 5 --warmup 1 --verbose"),
    "pmc_lzo41_lds": (300, "UDA_DECODE_WINDOW=lds timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS "
                           "SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv "
                           "-d gpurun_out/pmc_lzo41_lds -o run -- python3 bench.py --api --api-codec lzo --rows-per-gpu 100000000 "
                           "--steps 1 --warmup 0"),
    "ipc8_detail": (700, f"{PY} bench.py --gpus 8 --one-gpu --exchange ipc --rows-per-gpu 240000000 --steps 2 --warmup 1"),
    "nodefiles10_store3": (400, f"{PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 100000000 "
                                f"--provider-hbm-gb 3 --steps 1 --warmup 1"),
    "nodefiles10": (400, f"{PY} bench.py --api --node --mof-dir /tmp --reducers 15 --rows-per-gpu 100000000 --steps 1 --warmup 1"),
    "lzo130x5_reg": (600, f"UDA_DECODE_WINDOW=reg {PY} bench.py --api --api-codec lzo --steps 5 --warmup 1 --verbose"),
    "pmc_lzo41_lean": (300, "timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS "
                            "SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv "
                            "-d gpurun_out/pmc_lzo41_lean -o run -- python3 bench.py --api --api-codec lzo --rows-per-gpu 100000000 "
                            "--steps 1 --warmup 0"),
    "hybrid41b_s3": (700, "UDA_API_CONF=mapred.uda.gpu.hbm.budget=10000000000 "
                          f"{PY} bench.py --api --api-host-mofs --reducers 1 --rows-per-gpu 400000000 --steps 3 --warmup 1"),
    "store_tests": (300, f"{PY} -m pytest tests/test_gpu_api_device.py tests/test_gpu_mof_store.py -m gpu -x -v --timeout 170 "
                         f"--timeout-method thread -k 'hbm_store or mof_store or evict or holders or release'"),
    "prof_device_only": (400, "rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_device_only -o run -- "
                              "python3 bench.py --device-only --rows-per-gpu 400000000 --steps 2 --warmup 1"),
}

# PMC passes over one short device-only step: each pass stays within the per-block counter limits
PMC_PROG = "python3 bench.py --device-only --rows-per-gpu 100000000 --steps 1 --warmup 0 --no-validate"
PMC_PASSES = [
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES",
    "FETCH_SIZE",
    "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum",
]
for i, counters in enumerate(PMC_PASSES):
    RECIPES[f"pmc{i + 1}"] = (90, f"rocprofv3 --pmc {counters} --output-format csv -d gpurun_out/pmc{i + 1} -o run -- {PMC_PROG}")
# the K-way kernel against a plain device copy of the same bytes (tools/hbm_copy_roof.py): L2 traffic
# and hit rates per pass, each within the TCC block's 4 counters
ROOF_PASSES = {"a": "FETCH_SIZE TCC_HIT_sum", "b": "WRITE_SIZE TCC_MISS_sum",
               "c": "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
# raw L2 -> fabric read requests by size (FETCH_SIZE's derivation is checked against a copy of known bytes)
ROOF_PASSES["d"] = "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum"
for k, counters in ROOF_PASSES.items():
    RECIPES[f"roof_kws_{k}"] = (90, f"UDA_KWAY_STAGED=1 rocprofv3 --pmc {counters} --output-format csv -d gpurun_out/roof_kws_{k} "
                                    f"-o run -- {PMC_PROG}")
    RECIPES[f"roof_kw_{k}"] = (90, f"rocprofv3 --pmc {counters} --output-format csv -d gpurun_out/roof_kw_{k} -o run -- "
                                   f"{PMC_PROG}")
    RECIPES[f"roof_copy_{k}"] = (90, f"rocprofv3 --pmc {counters} --output-format csv -d gpurun_out/roof_copy_{k} -o run -- "
                                     f"python3 tools/hbm_copy_roof.py")


def summarize(path: str, keys: list[str]) -> str:
    line = None
    try:
        with open(path, errors="replace") as f:
            for ln in f:
                ln = ln.strip()
                if ln.startswith("{") and ln.endswith("}"):
                    line = ln
    except OSError:
        return ""
    if line is None:
        return ""
    try:
        d = json.loads(line)
    except ValueError:
        return line[:200]
    out = {k: d.get(k) for k in ["value", "validated", "ms_per_step", *keys] if k in d}
    return json.dumps(out)


def run_step(tag: str, name: str, seconds: int, cmd: str, keys: list[str]) -> int:
    os.makedirs(OUT, exist_ok=True)
    log = os.path.join(OUT, f"{tag}_{name}.log")
    err = os.path.join(OUT, f"{tag}_{name}.err")
    env = dict(os.environ, PYTHONUNBUFFERED="1", TMPDIR="/tmp")
    t0 = time.time()
    print(f"== {name} ({seconds}s): {cmd}", flush=True)
    with open(log, "w") as fo, open(err, "w") as fe:
        p = subprocess.Popen(["bash", "-c", cmd], cwd=ROOT, stdout=fo, stderr=fe, env=env, start_new_session=True)
        try:
            rc = p.wait(timeout=seconds)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGTERM)
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
            rc = 124
    dt = time.time() - t0
    s = summarize(log, keys)
    print(f"   rc={rc} {dt:.0f}s {s}", flush=True)
    if rc != 0:
        for path in (log, err):
            try:
                with open(path, errors="replace") as f:
                    tail = f.readlines()[-25:]
                print(f"   --- tail {os.path.basename(path)}", *tail, sep="   ", flush=True)
            except OSError:
                pass
    return rc


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("steps", nargs="*", help="recipe names, in order: " + " ".join(RECIPES))
    ap.add_argument("--tag", default="run", help="log file prefix under gpurun_out/")
    ap.add_argument("--cmd", action="append", default=[], help="ad-hoc step NAME=SECONDS=COMMAND")
    ap.add_argument("--keys", default="", help="extra JSON keys to print from each step's last JSON line")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_intermixed_args()  # steps may follow --cmd
    recipes = dict(RECIPES)
    for c in a.cmd:
        name, secs, cmd = c.split("=", 2)
        recipes[name] = (int(secs), cmd)
    if a.list:
        for k, (t, c) in recipes.items():
            print(f"{k:18s} {t:4d}s  {c}")
        return 0
    keys = [k for k in a.keys.split(",") if k]
    for name in a.steps:
        if name not in recipes:
            print(f"unknown step {name}", file=sys.stderr)
            return 2
        t, cmd = recipes[name]
        rc = run_step(a.tag, name, t, cmd, keys)
        if rc != 0:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
