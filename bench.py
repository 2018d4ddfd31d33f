#!/usr/bin/env python3
"""bench.py -- exact k=10 flat-index search throughput on MI355X.

Workload (BASELINE.json configs[2], the config north_star's target is quoted
on): 10M x 768 fp32 vectors, cosine ("cosine-dot"), k = 10, corpus sharded
over the N GPUs of one node by contiguous doc-id ranges (N=1: the whole 10M
corpus on one GPU).  One step = one batch of B = 8192 queries through the
full SearchByVector pipeline (query normalisation, bf16 block-key MFMA pass,
candidate-block selection, exact-order distances of the candidate rows,
exactness proof, bounded heap replay of any flagged query; for N>1 the
two-phase sharded search of the multi-shard index (multi.hip): RCCL all-gathers of the
block-key bounds and of the packed lists, the on-device merge and the
parallel cross-shard replay).  Inputs are synthetic (counter-based generator,
identical on CPU and GPU) and resident in HBM before timing starts.
--workload c1 / c2 run BASELINE configs[0] / [1] the same way.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "exact kNN QPS (k=10) at 1/2/4/8 GPUs; % of HBM-BW or MFMA roofline"
N_TOTAL = 10_000_000
DIMS = 768
K = 10
SEED_CORPUS = 1
SEED_QUERY = 2
MFMA_F32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
# exact flat workloads: BASELINE configs[0] (c1), [1] (c2), [2] (c3, the headline)
FLAT = {
    "c1": dict(n=100_000, d=128, metric="l2-squared", k=10, batch=1000, kind=0,
               name="Flat index exact kNN, 100k x 128 U(-1,1) fp32, l2-squared, k=10, 1k queries (BASELINE configs[0])"),
    "c2": dict(n=1_000_000, d=128, metric="l2-squared", k=100, batch=10_000, kind=1,
               name="SIFT-shaped 1M x 128 integer-valued fp32 U{0..127}, l2-squared, k=100, 10k-query batch "
                    "(BASELINE configs[1])"),
    # c3: 8192 queries per step -- one block-key launch of 32 query groups per
    # corpus span, every XCD's 32 workgroups on one span (60 % of the bf16 peak
    # vs 58 % at 4096 and 55 % at 2048) and the fixed per-step costs amortised
    # for the 8-GPU strong scaling
    "c3": dict(n=10_000_000, d=768, metric="cosine", k=10, batch=8192, kind=0,
               name="10M x 768 fp32 cosine, k=10, exact flat search (BASELINE configs[2])"),
}
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (spec, MI355X_MICROARCH.md)
MFMA_I8_PEAK_TOPS = 5000.0      # MI355X dense int8 MFMA: 2x bf16 per clock (MI355X_MICROARCH.md, Matrix cores)
# wv_stats.last_route (include/wv_knn.h WV_ROUTE_*) -> the dominant key kernel
ROUTE_KERNEL = {1: "k_qs_blockkey", 2: "k_qs_blockkey_w4", 3: "k_q8_blockkey", 4: "k_mfma_select3", 5: "k_gemv_select",
                9: "k_q8_gemv"}
# 32-bit integer VALU lane-ops/s: 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz.  The
# 32-lane/clk rate (78.6 T) is the f32 FMA rate; v_xor_b32 / v_bcnt_u32_b32 issue
# at 4 cycles per wave64 (measured: k_bq_blockmin_lds sustains 33.6 T instr-lane-ops/s).
VALU_PEAK_TOPS = 39.3
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
GEMV_MAX = 8                   # runtime.hip default "gemv_max": batches up to 8 queries take k_gemv_select

# BASELINE configs[3]: BQ 50M x 1536 over 8 GPUs -> one GPU holds a 6.25M-row shard
BQ_ROWS_PER_GPU = 6_250_000
BQ_DIMS = 1536
BQ_RESCORE = 200

# BASELINE configs[4]: PQ GIST-shaped 10M x 960, 240 segments x 256 centroids,
# k-means trained on a 100k sample, ADC search
PQ_ROWS = 10_000_000
PQ_DIMS = 960
PQ_SEGMENTS = 240
PQ_ADC_DEFAULT = "2"  # the index default of option pq_adc3 (rt_index.h): 2 = k_pq_adc4
PQ_CENTROIDS = 256
PQ_TRAIN = 100_000
# 4-byte LUT lookups from LDS: the LDS array moves 256 B/clk/CU (ds_read_b64 /
# b128; MI355X_MICROARCH.md LDS table) -> 64 lookups/clk/CU x 256 CU x 2.4 GHz;
# ds_read_b32 (one lookup per lane) is capped at half that (128 B/clk)
LDS_LOOKUP_PEAK_T = 39.3
LDS_LOOKUP_B32_T = 19.7


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return None


def host_info() -> dict:
    """nproc (CPUs this process may run on), the cgroup CPU quota, the CPU
    model, and the kernel variant the reference would pick on this host:
    AVX-512 only with AMX-BF16 && AVX512 (distancer/l2_amd64.go:19-26), else AVX2."""
    nproc = len(os.sched_getaffinity(0))
    model, flags = "", ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name") and not model:
                model = line.split(":", 1)[1].strip()
            if line.startswith("flags") and not flags:
                flags = line + " "
    except OSError:
        pass
    variant = "avx512" if (" amx_bf16 " in flags and " avx512f " in flags) else "avx256"
    return {"nproc": nproc, "cgroup_cpus": cgroup_cpus(), "cpu_model": model, "variant": variant}


def cpu_baseline(n_sample: int, nq: int, threads: int, spec=None):
    """Reference CPU flat scan on the host cores: the reference's own SIMD
    kernels (oracle/_ref, compiled from /root/reference) when the host can run
    them, else the oracle's scalar restatement; one query per thread, the
    kernel variant the reference's dispatch rule picks on this host."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # test infrastructure, used only for this baseline leg
    spec = spec or FLAT["c3"]
    info = host_info()
    use_ref = orc.ref_lib() is not None and orc.host_has_avx512()
    d, k, kind = spec["d"], spec["k"], spec["kind"]
    metric = orc.METRIC[spec["metric"]]
    variant = orc.AVX512 if info["variant"] == "avx512" else orc.AVX256
    corpus = orc.gen_matrix(kind, SEED_CORPUS, 0, n_sample, d)
    queries = orc.gen_matrix(kind, SEED_QUERY, 0, nq, d)
    if metric == orc.COSINE:
        orc.lib().or_normalize_rows(orc.f(corpus), n_sample, d)
        orc.lib().or_normalize_rows(orc.f(queries), nq, d)
    t0 = time.perf_counter()
    orc.cpu_baseline(metric, variant, corpus, queries, k, threads, use_ref)
    dt = time.perf_counter() - t0
    qps_sample = nq / dt
    # the scan is linear in N: extrapolate to the full corpus
    qps_full = qps_sample * n_sample / spec["n"]
    kname = ("l2" if metric == orc.L2 else "dot") + ("_512" if variant == orc.AVX512 else "_256")
    # the reference ships both SIMD variants: time the other one
    # too where this host can run it (AVX-512 needs the host's support)
    other = orc.AVX256 if variant == orc.AVX512 else orc.AVX512
    other_line = None
    if other == orc.AVX256 or orc.host_has_avx512():
        t1 = time.perf_counter()
        orc.cpu_baseline(metric, other, corpus, queries, k, threads, use_ref)
        dt1 = time.perf_counter() - t1
        other_line = {"variant": "avx512" if other == orc.AVX512 else "avx256",
                      "kernel": ("l2" if metric == orc.L2 else "dot") + ("_512" if other == orc.AVX512 else "_256"),
                      "value": nq / dt1 * n_sample / spec["n"], "seconds": round(dt1, 2)}
    return {
        "value": qps_full,
        "unit": "queries/s",
        "cores": threads,
        "kind": "reference" if use_ref else "port",
        "nproc": info["nproc"],
        "cgroup_cpus": info["cgroup_cpus"],
        "cpu_model": info["cpu_model"],
        "variant": info["variant"],
        "other_variant": other_line,
        "sample": (f"{nq} queries x {n_sample} rows (first rows of the same corpus), {spec['metric']} k={k}, "
                   f"{'reference ' + kname + ' kernel (oracle/_ref)' if use_ref else 'oracle scalar restatement'} "
                   f"+ NewMax heap scan, {threads} threads, {dt:.1f} s"
                   + (f", QPS scaled by {n_sample}/{spec['n']}" if n_sample != spec["n"] else "")),
    }


def cpu_baseline_bq(n_sample: int, nq: int, threads: int, n_full: int):
    """Reference CPU BQ flat search (searchByVectorQuantized restated in
    oracle/baseline.c) with the reference's own hamming_bitwise_256 and dot_256
    kernels (oracle/_ref) when the host can run them; one query per thread."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # test infrastructure, used only for this baseline leg
    use_ref = orc.ref_lib() is not None and orc.host_has_avx512()
    corpus = orc.gen_matrix(0, SEED_CORPUS, 0, n_sample, BQ_DIMS)
    orc.lib().or_normalize_rows(orc.f(corpus), n_sample, BQ_DIMS)
    words = (BQ_DIMS + 63) // 64
    bits = np.zeros((n_sample, words * 64), dtype=bool)
    bits[:, :BQ_DIMS] = corpus < 0
    codes = np.packbits(bits, axis=1, bitorder="little").view("<u8").reshape(n_sample, words)
    queries = orc.gen_matrix(0, SEED_QUERY, 0, nq, BQ_DIMS)
    orc.lib().or_normalize_rows(orc.f(queries), nq, BQ_DIMS)
    t0 = time.perf_counter()
    orc.cpu_baseline_bq(orc.COSINE, orc.AVX256, corpus, codes, queries, K, BQ_RESCORE, threads, use_ref)
    dt = time.perf_counter() - t0
    return {
        "value": nq / dt * n_sample / n_full,
        "unit": "queries/s",
        "cores": threads,
        "kind": "reference" if use_ref else "port",
        "sample": (f"{nq} queries x {n_sample} rows, BQ hamming R={BQ_RESCORE} heap + fp32 rescoring, "
                   f"{'reference hamming_bitwise_256 + dot_256 kernels (oracle/_ref)' if use_ref else 'oracle scalar restatement'}, "
                   f"{dt:.1f} s, QPS scaled by {n_sample}/{n_full}"),
    }


def cpu_baseline_pq(index, n_sample: int, nq: int, threads: int, n_full: int):
    """CPU PQ flat search (oracle/baseline.c: DistanceLookUpTable + LookUp +
    flatSearch heap, restated) on the same codebook and codes; one query per
    thread.  There is no reference kernel to call: the Go LookUp loop is pure Go."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # test infrastructure, used only for this baseline leg
    centers = index.pq_centers()
    codes = index.pq_codes(n_sample)
    queries = orc.gen_matrix(2, SEED_QUERY, 0, nq, PQ_DIMS)
    t0 = time.perf_counter()
    orc.cpu_baseline_pq(orc.L2, centers, codes, queries, K, threads)
    dt = time.perf_counter() - t0
    return {
        "value": nq / dt * n_sample / n_full,
        "unit": "queries/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{nq} queries x {n_sample} rows, LUT + ADC (m={PQ_SEGMENTS}) + heap, oracle C restatement, "
                   f"{dt:.1f} s, QPS scaled by {n_sample}/{n_full}"),
    }


def cpu_baseline_rq(bits: int, n_sample: int, nq: int, threads: int, n_full: int):
    """CPU rq-8 / rq-1 flat search (oracle/rq.c restating flat.searchByVectorQuantized
    with the rotational quantizers) on the first n_sample rows of the same
    corpus, one query per thread (ctypes releases the GIL)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # test infrastructure, used only for this baseline leg
    from concurrent.futures import ThreadPoolExecutor
    corpus = orc.gen_matrix(0, SEED_CORPUS, 0, n_sample, DIMS)
    flat = orc.OracleFlatRQ(bits, orc.COSINE, orc.AVX256, DIMS, n_sample, BQ_RESCORE)
    flat.add_batch(np.arange(n_sample, dtype=np.uint64), corpus)
    queries = orc.gen_matrix(0, SEED_QUERY, 0, nq, DIMS)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda i: flat.search(queries[i], K), range(nq)))
    dt = time.perf_counter() - t0
    return {
        "value": nq / dt * n_sample / n_full,
        "unit": "queries/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{nq} queries x {n_sample} rows, rq-{bits} R={BQ_RESCORE} heap + fp32 rescoring, oracle C "
                   f"restatement (oracle/rq.c), {dt:.1f} s, QPS scaled by {n_sample}/{n_full}"),
    }


def verify_sample(workload: str, flat, gen_kind: int, n_total: int, dims: int, B: int, k: int, res, index,
                  threads: int, bq_r: int = 0, world: int = 1):
    """The bench checks its own output: a sample of the step's result rows
    (16 queries spread over the batch; 8 for PQ) against the oracle's exact
    scan of the regenerated corpus (oracle/scale.c; the reference heap
    semantics of flat/index.go:578-688), bit-exact ids and distances.
    rq-8 / rq-1: oracle/scale.c's or_rq_search_gen encodes every regenerated
    row on the host (rq.c's rotation + encoder) and replays the R-heap per
    sampled query.  Returns {"verified": bool, "checked": n, ...} or None when
    the workload has no oracle check here."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # test infrastructure: the checker, outside the timed region
    ids, dists, counts = (t.cpu().numpy() for t in res)
    ids = ids.view(np.uint64)
    t0 = time.perf_counter()
    nchk = 8 if workload == "pq" else 16
    sample = np.unique(np.linspace(0, B - 1, nchk).astype(np.int64))
    bad = []
    if flat is not None:
        metric = orc.METRIC[flat["metric"]]
        qs = orc.gen_matrix(gen_kind, SEED_QUERY, 0, B, dims)[sample]
        if metric == orc.COSINE:
            qs = np.stack([orc.normalize(x) for x in qs])
        D = orc.gen_dists(gen_kind, SEED_CORPUS, n_total, dims, metric, orc.AVX256, qs, threads)
        exp = [orc.heap_scan(D[i], k) for i in range(len(sample))]
        del D
    elif workload == "bq":
        qs = orc.gen_matrix(0, SEED_QUERY, 0, B, dims)[sample]
        oi, od, on = orc.bq_search_gen(0, SEED_CORPUS, n_total, dims, orc.COSINE, orc.AVX256, qs, k, bq_r, threads)
        exp = [(oi[i, :on[i]], od[i, :on[i]]) for i in range(len(sample))]
    elif workload in ("rq8", "rq1"):
        qs = orc.gen_matrix(gen_kind, SEED_QUERY, 0, B, dims)[sample]
        oi, od, on = orc.rq_search_gen(8 if workload == "rq8" else 1, gen_kind, SEED_CORPUS, n_total, dims, orc.COSINE,
                                       orc.AVX256, qs, k, bq_r, threads)
        exp = [(oi[i, :on[i]], od[i, :on[i]]) for i in range(len(sample))]
    elif workload == "pq" and world == 1:
        from concurrent.futures import ThreadPoolExecutor
        centers, codes = index.pq_centers(), index.pq_codes(n_total)
        present = np.ones(n_total, np.uint8)
        dummy = np.zeros(1, np.float32)
        qs = orc.gen_matrix(2, SEED_QUERY, 0, B, dims)[sample]
        with ThreadPoolExecutor(min(threads, len(sample))) as ex:
            exp = list(ex.map(lambda i: orc.pq_flat_search(orc.L2, orc.AVX256, centers, codes, dummy, present, qs[i],
                                                           k, k, False), range(len(sample))))
        del codes
    else:
        return None
    for i, q in enumerate(sample):
        ei, ed = exp[i]
        c = int(counts[q])
        if c != len(ei) or not np.array_equal(ids[q, :c], np.asarray(ei, np.uint64)) or \
                not np.array_equal(np.asarray(dists[q, :c], np.float32).view(np.uint32),
                                   np.asarray(ed, np.float32).view(np.uint32)):
            bad.append(int(q))
    return {"verified": not bad, "checked_queries": [int(x) for x in sample], "mismatched": bad,
            "against": "oracle exact scan of the regenerated corpus (bit-exact ids and distances)",
            "seconds": round(time.perf_counter() - t0, 1)}


def measured_traffic(workload: str, n_local: int, dims: int, batch: int, kernel: str = None):
    """HBM bytes per launch of `kernel` from a committed PMC pass
    (profiles/*_pmc_*.json, tools/pmc_traffic.sh) taken on this exact
    configuration and kernel; None otherwise."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_*.json"))):
        try:
            rec = json.load(open(path))
        except Exception:
            continue
        if (rec.get("corpus_rows"), rec.get("dims"), rec.get("query_batch"), rec.get("kernel")) == \
                (n_local, dims, batch, kernel):
            best = rec.get("hbm_bytes_per_launch")
    return best


def measured_clock(workload: str, n_local: int, dims: int, batch: int, kernel: str):
    """Effective clock and MFMA-busy fraction of the dominant kernel from the
    committed PMC record (profiles/*_clock_<workload>*.json, tools/pmc_qs3.sh)
    when it was taken on this exact configuration; None otherwise."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", f"*_clock_{workload}*.json"))):
        try:
            rec = json.load(open(path))
        except Exception:
            continue
        if (rec.get("corpus_rows"), rec.get("dims"), rec.get("query_batch"), rec.get("kernel")) == \
                (n_local, dims, batch, kernel):
            best = {k: rec[k] for k in ("effective_clock_ghz", "mfma_busy_frac", "frac_of_peak_at_clock")}
            best["source"] = os.path.relpath(path, REPO)
    return best


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def relaunch_cmd(argv, n: int, port: int):
    """`python -m torch.distributed.run` over N local ranks running this same
    bench.py with the same arguments (one process per GPU, rendezvous on
    127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def maybe_relaunch(argv, gpus: int, env=None, run=None) -> int | None:
    """--gpus N > 1 without a launcher (no WORLD_SIZE in the environment): start
    the N-rank run as a child process -- before this process touches the GPU
    (nothing here imports torch) -- relay its output and return its exit code.
    None: no relaunch (a single GPU, or already one rank of a launcher)."""
    env = os.environ if env is None else env
    if gpus <= 1 or "WORLD_SIZE" in env:
        return None
    import subprocess
    run = run or subprocess.run
    cmd = relaunch_cmd(argv, gpus, free_port())
    log("[bench] --gpus %d without a launcher: %s" % (gpus, " ".join(cmd)))
    child_env = dict(env)
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = run(cmd, env=child_env, stdout=subprocess.PIPE, text=True)
    for line in (p.stdout or "").splitlines():
        if line.startswith("{"):  # rank 0's JSON line
            print(line, flush=True)
    return p.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c3", "c1", "c2", "bq", "pq", "rq8", "rq1"], default="c3",
                    help="c3: 10M x 768 cosine exact (default, the headline); c1 / c2: BASELINE configs[0] / [1]; "
                         "bq: BQ 1536-d shard of configs[3]; "
                         "pq: configs[4] PQ 10M x 960 (k-means fit timed once, ADC search timed per step); "
                         "rq8 / rq1: flat's rotational quantizers on the c3 corpus, R=200 rescoring")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--rows", "--n", dest="n", type=int, default=None,
                    help="corpus rows (--rows under torch.distributed.run: its parser claims --n as a prefix)")
    ap.add_argument("--dims", type=int, default=None,
                    help="exact flat workloads: override the row width (e.g. 1024 / 1536, the block-key w4 kernel)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--option", action="append", default=[],
                    help="index option key=value (wv_index_set_option), e.g. qs_w4=1; repeatable")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the self-check of sampled result rows against the oracle (outside the timed region)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the multi-GPU path (the multi-shard index over RCCL, multi.hip) even at WORLD_SIZE 1 "
                         "(launch under torch.distributed.run): a one-GPU check of the N>1 path")
    ap.add_argument("--cpu-rows", type=int, default=1_000_000)
    ap.add_argument("--cpu-queries", type=int, default=None)
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: nproc (all CPUs this process may use)")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per k_mfma_select launch from the rocprofv3 PMC pass")
    args = ap.parse_args()
    rc = maybe_relaunch(sys.argv[1:], args.gpus)
    if rc is not None:
        sys.exit(rc)
    if args.cpu_threads is None:
        # every CPU this process may use: nproc, capped by a cgroup quota (more
        # threads than the quota only time-slice the same cores)
        quota = cgroup_cpus()
        args.cpu_threads = len(os.sched_getaffinity(0)) if quota is None else min(quota, len(os.sched_getaffinity(0)))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch one rank per GPU "
                         "(bench.py starts torch.distributed.run itself when WORLD_SIZE is unset)")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    shard = world > 1 or args.sharded
    if shard:
        dist.init_process_group("nccl", device_id=dev)

    import weaviate_amd as wv
    from weaviate_amd import _lib
    lib = _lib.load()

    bq = args.workload == "bq"
    pq = args.workload == "pq"
    rq_bits = {"rq8": 8, "rq1": 1}.get(args.workload, 0)
    flat = FLAT.get(args.workload)  # exact fp32 flat search (c1 / c2 / c3)
    if flat is not None and args.dims is not None and args.dims != flat["d"]:
        flat = dict(flat, d=args.dims, name=flat["name"].replace(f"x {flat['d']} ", f"x {args.dims} ")
                    + f" at d={args.dims}")
    dims = BQ_DIMS if bq else PQ_DIMS if pq else flat["d"] if flat else DIMS
    K_ = flat["k"] if flat else K
    # flat / pq: a fixed corpus split over the ranks (strong scaling); bq: configs[3]
    # is 50M rows over 8 GPUs, i.e. a 6.25M-row shard per GPU (weak scaling)
    n_total = args.n if args.n is not None else (BQ_ROWS_PER_GPU * world if bq else PQ_ROWS if pq
                                                 else flat["n"] if flat else N_TOTAL)
    n_local = (n_total + world - 1) // world
    id0 = rank * n_local
    n_local = max(0, min(n_local, n_total - id0))
    # pq: 2048 queries per step (the int8 key pass is MFMA-bound from ~1k queries; 256 keeps it HBM-bound)
    B = args.batch if args.batch is not None else (2048 if pq else flat["batch"] if flat else 2048)
    # GIST-shaped U[0,1) for PQ, SIFT-shaped integers for c2, U[-1,1) otherwise
    gen_kind = 2 if pq else flat["kind"] if flat else 0
    metric_name = "l2-squared" if pq else flat["metric"] if flat else "cosine"

    # ---- build the shard: generate + add in 1M-row chunks (device resident) ----
    t_build = time.perf_counter()
    multi = None
    comp = dict(bq=bq, rescore_limit=BQ_RESCORE if (bq or rq_bits) else -1, rq={"bits": rq_bits} if rq_bits else None,
                pq={"segments": PQ_SEGMENTS, "centroids": PQ_CENTROIDS, "trainingLimit": PQ_TRAIN,
                    "rescore": False} if pq else None)
    if shard:
        # the search over N GPUs: the library's multi-shard index (multi.hip)
        # drives the protocol of the workload's kind (exact two-phase block keys,
        # BQ R-heap, PQ / rq worker heap) and owns an RCCL communicator; rank 0's
        # unique id reaches every process over the launcher's process group
        from weaviate_amd.sharded import open_multi
        multi = open_multi(n_total, local_rank, distance=metric_name, dims=dims, variant="avx256", **comp)
        index = multi.shards[0]
    else:
        index = wv.FlatIndex(distance=metric_name, dims=dims, device=local_rank, variant="avx256", id_base=id0, **comp)
    for kv in args.option:
        key, val = kv.split("=", 1)
        index.set_option(key, int(val))
    index.reserve(n_local)
    chunk = 1_000_000
    stage = torch.empty((min(chunk, max(n_local, 1)), dims), dtype=torch.float32, device=dev)
    for r0 in range(0, n_local, chunk):
        m = min(chunk, n_local - r0)
        _lib.check(lib.wv_gen_device(local_rank, gen_kind, SEED_CORPUS, id0 + r0, m, dims, stage.data_ptr(), None))
        _lib.check(lib.wv_index_add_range_device(index._h, id0 + r0, stage.data_ptr(), m, dims))
    del stage
    queries = torch.empty((B, dims), dtype=torch.float32, device=dev)
    _lib.check(lib.wv_gen_device(local_rank, gen_kind, SEED_QUERY, 0, B, dims, queries.data_ptr(), None))
    torch.cuda.synchronize()
    log(f"[rank {rank}] shard ids [{id0}, {id0 + n_local}) built in {time.perf_counter() - t_build:.1f} s")
    fit_s = None
    if pq:
        torch.cuda.synchronize()
        t_fit = time.perf_counter()
        if shard and n_local < PQ_TRAIN:
            # the single index trains on the first trainingLimit rows of the whole corpus: rank 0 must hold them
            raise SystemExit(f"sharded PQ needs >= {PQ_TRAIN} rows on rank 0 (has {n_local})")
        if shard:  # rank 0 holds ids [0, n_local): it trains, the codebook goes to every shard over RCCL
            multi.pq_fit(seed=SEED_CORPUS)
        else:
            index.pq_fit(seed=SEED_CORPUS)
        torch.cuda.synchronize()
        fit_s = time.perf_counter() - t_fit
        log(f"[rank {rank}] pq fit ({PQ_SEGMENTS} x k-means k={PQ_CENTROIDS} on {PQ_TRAIN} rows) + encode "
            f"{n_local} rows: {fit_s:.2f} s")
    index.set_option("timing", 1)

    out_ids = torch.empty((B, K_), dtype=torch.int64, device=dev)
    out_d = torch.empty((B, K_), dtype=torch.float32, device=dev)
    out_n = torch.empty(B, dtype=torch.int32, device=dev)

    if shard:
        def step():
            s = torch.cuda.current_stream(dev).cuda_stream
            multi.search_device(queries.data_ptr(), B, dims, K_, out_ids.data_ptr(), out_d.data_ptr(),
                                out_n.data_ptr(), s)
            return out_ids, out_d, out_n
    else:
        def step():
            s = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(lib.wv_index_search_device(index._h, queries.data_ptr(), B, dims, K_, 0, out_ids.data_ptr(),
                                                  out_d.data_ptr(), out_n.data_ptr(), None, s))
            return out_ids, out_d, out_n

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    sel_ms, tot_ms = [], []
    replays0 = index.stats()["replayed_queries"]
    flagged0 = multi.stats()["flagged"] if multi is not None else 0
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
        st = index.stats()
        sel_ms.append(st["last_select_ms"])
        tot_ms.append(st["last_total_ms"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    replays = index.stats()["replayed_queries"] - replays0
    route = int(index.stats().get("last_route", 0))
    if multi is not None:
        replays = multi.stats()["flagged"] - flagged0  # the cross-shard replay's queries (every rank's view)
    sharded_check = None
    if args.sharded and world == 1:
        # the sharded protocol at one rank must equal the single-index search
        si, sd, sn = (t.clone() for t in step()[:3])
        s = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.wv_index_search_device(index._h, queries.data_ptr(), B, dims, K_, 0, out_ids.data_ptr(),
                                              out_d.data_ptr(), out_n.data_ptr(), None, s))
        torch.cuda.synchronize()
        sharded_check = bool(torch.equal(sn, out_n) and torch.equal(si.view(torch.int64), out_ids)
                             and torch.equal(sd.view(torch.int32), out_d.view(torch.int32)))
        log(f"sharded protocol at world 1 equals the single-index search: {sharded_check}")
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        sm = torch.tensor([float(np.mean(sel_ms))], dtype=torch.float64, device=dev)
        dist.all_reduce(sm, op=dist.ReduceOp.MAX)
        sel_avg = float(sm.item())
    else:
        sel_avg = float(np.mean(sel_ms))

    total_q = B * args.steps
    value = total_q / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # the exact fp32 path's dominant kernel: the block-key pass the runtime chose
    # (int8 keys for 384 < d <= 1536, bf16 keys otherwise; wv_stats.last_route)
    sel_kernel = ROUTE_KERNEL.get(route, "k_qs_blockkey")
    if route == 3 and dims > 1536:  # int8-only planes: the two-column-part form
        sel_kernel = "k_q8_blockkey_cp"
    int8_keys = sel_kernel.startswith("k_q8_")
    total_avg = float(np.mean(tot_ms)) if tot_ms else 0.0
    # the dominant kernel of each workload: its PMC record (matched on kernel
    # name and configuration) is the only source of `traffic`
    # the sharded PQ search (the multi-shard worker heap, wv_index_quant_*) computes full ADC rows with k_pq_adc2
    pq_opt = [o.replace(" ", "") for o in args.option if o.replace(" ", "").startswith("pq_adc3=")]
    pq_sel = pq_opt[-1].split("=")[1] if pq_opt else PQ_ADC_DEFAULT
    pq_kernel = ("k_q8_blockkey_pq" if route == 8 else
                 "k_pq_adc2" if shard or pq_sel == "0" else "k_pq_adc4" if pq_sel == "2" else "k_pq_adc3") if pq \
        else "k_pq_adc2"
    dom_kernel = (pq_kernel if pq else ("k_q8_blockkey_bq" if route == 6 else "k_bq_blockmin_lds") if bq else
                  ("k_rq8_keys" if route == 10 else "k_rq8_dist" if rq_bits == 8 else "k_rq1_dist") if rq_bits
                  else sel_kernel)
    if args.traffic_bytes is None:
        args.traffic_bytes = measured_traffic(args.workload, n_local, dims, B, dom_kernel)
    if rq_bits and route == 10:
        # dominant kernel: k_rq8_keys (rq8_mfma.hip), the
        # exact rq-8 distance of every (query, row) on v_mfma_i32_16x16x64_i8
        # (one int8 product per (query, row, code byte), D = dims rounded up to
        # 64) plus the reference's float epilogue, reduced to 32-row minima in
        # registers; the codes (n_local x D bytes) stream once per launch
        D = (dims + 63) // 64 * 64
        f0 = int(index.stats().get("last_group_queries", 0)) or B
        t = sel_avg * 1e-3
        ops = 2.0 * f0 * n_local * D
        plane = float(n_local) * (D + 20)
        mfma_frac = ops / t / 1e12 / MFMA_I8_PEAK_TOPS if t > 0 else 0.0
        hbm_frac = plane / t / 1e9 / HBM_PEAK_GBPS if t > 0 else 0.0
        roof = {"bound": "mfma", "kernel": "k_rq8_keys", "achieved": ops / t / 1e12 if t > 0 else 0.0,
                "peak": MFMA_I8_PEAK_TOPS, "unit": "TOPS (int8 MFMA)", "frac": mfma_frac, "launch_ms": sel_avg,
                "hbm_frac": hbm_frac,
                "algorithmic": f"2 x {f0} x {n_local} x {D} int8 ops; {n_local} x {D + 20} code + meta bytes",
                "mfma": "v_mfma_i32_16x16x64_i8 on (x - 128)(y - 128) + 128 (Sx + Sy) - 16384 D = dotByteImpl "
                        "exactly; the reference's fp32 epilogue per (query, row), unfused",
                "epilogue_valu_per_pair": "about 17 VALU ops per (query, row): the kernel is VALU-issue bound",
                "traffic": args.traffic_bytes}
    elif rq_bits:
        # dominant kernel k_rq8_dist / k_rq1_dist, timed on the first query
        # group of the batch (search_rq: groups of RQ_QPB multiples whose
        # distance rows fit 4 GiB).  rq-8: one v_dot4_u32_u8 per 4 code bytes
        # and (query, row); rq-1: per 64-bit word and (query, row) 5 bit planes
        # x (2 v_xor_b32 + 2 v_bcnt_u32_b32).  The kernel also writes the
        # 4-byte quantized distance of every (query, row) pair.
        D = (dims + 63) // 64 * 64
        ld = max((n_local + 255) // 256 * 256, 256)
        f0 = int(index.stats().get("last_group_queries", 0)) or min(B, max(32, ((4 << 30) // (ld * 4)) // 32 * 32))
        ops = float(f0) * n_local * (D / 4 if rq_bits == 8 else (D / 64) * 5 * 4)
        achieved = ops / (sel_avg * 1e-3) / 1e12 if sel_avg > 0 else 0.0
        kname = "k_rq8_dist" if rq_bits == 8 else "k_rq1_dist"
        roof = {"bound": "valu", "kernel": kname, "achieved": achieved, "peak": VALU_PEAK_TOPS,
                "unit": "Tops/s (int32 lane-ops)", "frac": achieved / VALU_PEAK_TOPS, "launch_ms": sel_avg,
                "note": f"launch_ms = first query group ({f0} queries) of the batch",
                "hbm_write_GBps": f0 * ld * 4 / (sel_avg * 1e-3) / 1e9 if sel_avg > 0 else 0.0,
                "traffic": args.traffic_bytes}
    elif pq and route == 8:
        # dominant kernel: the block keys on the integer matrix cores over the
        # centred int8 reconstruction plane (k_q8_blockkey):
        # one int8 product per (query, row, dim) and the plane (n_local x dpb8
        # bytes) streamed once per launch; the binding roofline is the larger
        # fraction (HBM at small batches, MFMA at large)
        dpb8 = (dims + 127) // 128 * 128 if dims <= 768 else (dims + 255) // 256 * 256
        f0 = int(index.stats().get("last_group_queries", 0)) or B
        t = sel_avg * 1e-3
        ops = 2.0 * f0 * n_local * dims
        plane = float(n_local) * dpb8
        mfma_frac = ops / t / 1e12 / MFMA_I8_PEAK_TOPS if t > 0 else 0.0
        hbm_frac = plane / t / 1e9 / HBM_PEAK_GBPS if t > 0 else 0.0
        if hbm_frac >= mfma_frac:
            roof = {"bound": "hbm", "kernel": pq_kernel, "achieved": plane / t / 1e9 if t > 0 else 0.0,
                    "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": hbm_frac}
        else:
            roof = {"bound": "mfma", "kernel": pq_kernel, "achieved": ops / t / 1e12 if t > 0 else 0.0,
                    "peak": MFMA_I8_PEAK_TOPS, "unit": "TOPS (int8 MFMA)", "frac": mfma_frac}
        roof.update({"launch_ms": sel_avg, "mfma_frac": mfma_frac, "hbm_frac": hbm_frac,
                     "algorithmic": f"2 x {f0} x {n_local} x {dims} int8 ops; {n_local} x {dpb8} plane bytes",
                     "mfma": "v_mfma_i32_16x16x64_i8 over the centred reconstruction x~ - mu (l2 keys; exact ADC "
                             "of the candidate rows from the LUT, reference segment order)",
                     "traffic": args.traffic_bytes})
    elif pq:
        # dominant kernel k_pq_adc4 (k_pq_adc3 / k_pq_adc2 with --option
        # pq_adc3=1 / 0): one LUT lookup (LDS read) + fp32 add per (query, row,
        # segment); adc4 reads 64 queries' entries of four rows' codes per
        # ds_read_b128 (conflict-free), so the LDS array rate for 4-byte
        # lookups is the peak
        ld = (n_local + 255) // 256 * 256
        f0 = int(index.stats().get("last_group_queries", 0)) or max(1, min(B, (2 << 30) // (ld * 4)))  # timed first group
        lookups = float(f0) * n_local * PQ_SEGMENTS
        achieved = lookups / (sel_avg * 1e-3) / 1e12 if sel_avg > 0 else 0.0
        roof = {"bound": "lds", "kernel": pq_kernel, "achieved": achieved,
                "peak": LDS_LOOKUP_PEAK_T, "unit": "T lookups/s", "frac": achieved / LDS_LOOKUP_PEAK_T,
                "frac_of_b32_lookup_rate": achieved / LDS_LOOKUP_B32_T, "launch_ms": sel_avg,
                "note": "launch_ms = first query group of the batch",
                "traffic": args.traffic_bytes}
    elif bq and route == 6:
        # dominant kernel: the block minima on the integer matrix cores
        # (k_q8_blockkey<..., BQ> over the +-1 code planes): one int8 product
        # per (query, row, code bit), hamming = (bits - dot) / 2 exactly
        words = (dims + 63) // 64
        ops = 2.0 * B * n_local * 64 * words
        achieved = ops / (sel_avg * 1e-3) / 1e12 if sel_avg > 0 else 0.0
        roof = {"bound": "mfma", "kernel": "k_q8_blockkey (BQ +-1 planes)", "achieved": achieved,
                "peak": MFMA_I8_PEAK_TOPS, "unit": "TOPS (int8 MFMA)", "frac": achieved / MFMA_I8_PEAK_TOPS,
                "launch_ms": sel_avg,
                "mfma": "v_mfma_i32_16x16x64_i8 over codes unpacked to +-1 int8: sum s_q s_x = bits - 2 hamming",
                "valu_form_equivalent_Tops": 4.0 * B * n_local * words / (sel_avg * 1e-3) / 1e12 if sel_avg > 0 else 0.0,
                "traffic": args.traffic_bytes}
    elif bq:
        # dominant kernel k_bq_blockmin: VALU-bound integer work, per (query,
        # row) pair and 64-bit code word 2 v_xor_b32 + 2 v_bcnt_u32_b32
        words = (dims + 63) // 64
        ops = 4.0 * B * n_local * words
        achieved = ops / (sel_avg * 1e-3) / 1e12 if sel_avg > 0 else 0.0
        roof = {"bound": "valu", "kernel": "k_bq_blockmin_lds", "achieved": achieved, "peak": VALU_PEAK_TOPS,
                "unit": "Tops/s (int32 lane-ops)", "frac": achieved / VALU_PEAK_TOPS, "launch_ms": sel_avg,
                "hbm_GBps": n_local * words * 8 / (sel_avg * 1e-3) / 1e9 if sel_avg > 0 else 0.0,
                "traffic": args.traffic_bytes}
    else:
        # roofline of the dominant kernel (k_q8_blockkey, DESIGN.md 3.1f, or
        # k_qs_blockkey, 3.1d): one MFMA product per (query, row, dim):
        # algorithmic ops per launch = 2 * B * n_local * d, over its measured
        # average duration (HIP events on the stream it runs on), against the
        # dense peak of the MFMA's input type (int8: 5 POPS, bf16: 2.5 PFLOPS).
        # the timed launch is the first query chunk of the batch (search_qs)
        f0 = int(index.stats().get("last_group_queries", 0)) or B
        flops = 2.0 * min(B, f0) * n_local * dims
        achieved = flops / (sel_avg * 1e-3) / 1e12 if sel_avg > 0 else 0.0
        peak = MFMA_I8_PEAK_TOPS if int8_keys else MFMA_BF16_PEAK_TFLOPS
        roof = {"bound": "mfma", "kernel": sel_kernel, "achieved": achieved, "peak": peak,
                "unit": "TOPS (int8 MFMA)" if int8_keys else "TFLOP/s", "frac": achieved / peak, "launch_ms": sel_avg,
                "mfma": ("v_mfma_i32_16x16x64_i8 (int8 in, exact int32 accumulate; per-block / per-query scales)"
                         if int8_keys else
                         ("v_mfma_f32_16x16x32_bf16" if dims > 384 else "v_mfma_f32_32x32x16_bf16")
                         + " (bf16 in, fp32 accumulate)")
                        + ": block keys = per-32-row minima of the approximate distance; every returned "
                          "distance is the reference-order fp32 value",
                "pipeline_ms": total_avg,
                "traffic": args.traffic_bytes,
                # DVFS: the chip holds a lower clock under this MFMA load; the PMC
                # record gives the clock and the MFMA pipe's busy fraction
                "pmc_clock": measured_clock(args.workload, n_local, dims, B, sel_kernel)}

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:  # every world size: rank 0, outside the timed region
            try:
                if rq_bits:
                    cpu = cpu_baseline_rq(rq_bits, min(args.cpu_rows, 200_000), args.cpu_queries or 512,
                                          args.cpu_threads, n_total)
                elif pq:
                    cpu = cpu_baseline_pq(index, min(args.cpu_rows, n_total), args.cpu_queries or 256,
                                          args.cpu_threads, n_total)
                elif bq:
                    cpu = cpu_baseline_bq(min(args.cpu_rows, n_total), args.cpu_queries or 4096, args.cpu_threads,
                                          n_total)
                else:
                    spec = dict(flat)
                    spec["n"] = n_total
                    # c1 is small enough to time in full (every query, every row)
                    rows = n_total if args.workload == "c1" else min(args.cpu_rows, n_total)
                    nqc = args.cpu_queries or (B if args.workload == "c1" else 1024)
                    cpu = cpu_baseline(rows, nqc, args.cpu_threads, spec)
            except Exception as e:  # baseline failure must not hide the GPU number
                log(f"cpu baseline failed: {e}")
        check = None
        if not args.no_verify:
            try:
                check = verify_sample(args.workload, flat, gen_kind, n_total, dims, B, K_, res[:3], index,
                                      args.cpu_threads, BQ_RESCORE, world)
                if check is not None:
                    log(f"self-check: {check}")
            except Exception as e:
                check = {"verified": False, "error": repr(e)}
        if rq_bits:
            workload = (f"rq-{rq_bits} (flat rotational quantization) {dims}-d cosine, k={K}, rescore R={BQ_RESCORE}, "
                        f"on the BASELINE configs[2] corpus ({n_total} rows)")
        elif pq:
            workload = (f"PQ {dims}-d l2-squared, m={PQ_SEGMENTS} x ks={PQ_CENTROIDS} trained on {PQ_TRAIN} rows "
                        f"(fit {fit_s:.2f} s), ADC flat search k={K} (BASELINE configs[4])")
        elif bq:
            workload = (f"BQ {dims}-d cosine, k={K}, rescore R={BQ_RESCORE}: one {n_total}-row shard of "
                        "BASELINE configs[3] (50M x 1536 over 8 GPUs)")
        else:
            workload = flat["name"]
        result = {
            "metric": METRIC,
            "value": value,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak" if bq else "strong",
            "vs_baseline": None,
            "dtype": ("u8 codes (int8 MFMA, exact int32 dot) + f32 rescoring" if rq_bits == 8 and route == 10 else
                      "u8 codes (v_dot4) + f32 rescoring" if rq_bits == 8 else
                      "u64 codes x 5-bit query planes + f32 rescoring" if rq_bits == 1 else
                      "+-1 int8 codes (hamming on the integer MFMA) + f32 rescoring" if bq and route == 6 else
                      "u64 hamming + f32 rescoring" if bq else "u8 codes + f32 LUT" if pq else
                      "f32 (exact result; int8 MFMA block-key filter)" if int8_keys else
                      "f32 (exact result; bf16 MFMA block-key filter)"),
            "data": ("synthetic (counter-based integer U{0..127} generator, seed 1 corpus / 2 queries)" if gen_kind == 1
                     else "synthetic (counter-based U[0,1) generator, seed 1 corpus / 2 queries)" if gen_kind == 2
                     else "synthetic (counter-based U[-1,1) generator, seed 1 corpus / 2 queries)"),
            "config": {
                "workload": workload,
                "corpus_rows": n_total,
                "dims": dims,
                "k": K_,
                "query_batch": B,
                "parallelism": f"corpus sharded over {world} GPU(s), contiguous id ranges"
                               + ((", R-heap replay in one parallel hop (all-gathered block-minimum bounds, "
                                   "recorded insertions, on-device merge) + all-gather rescoring" if bq
                                   else ", worker heap in one parallel hop (block-minimum bounds, recorded "
                                   "insertions, on-device merge)" + (", codebook trained on rank 0 and broadcast" if pq
                                                                     else ", all-gather rescoring") if (pq or rq_bits)
                                   else ", multi-shard index (multi.hip): library-owned RCCL communicator, "
                                   "all-gathers of the block-key bounds and lists, on-device merge, parallel "
                                   "cross-shard replay") if world > 1 else ""),
                "replayed_queries": int(replays),
            },
            **({"sharded_equals_single": sharded_check} if sharded_check is not None else {}),
            "verified": None if check is None else check["verified"],
            "verify": check,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()  # the other ranks wait for rank 0's host legs
    index.close()
    if multi is not None:
        multi.close()
    if shard:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
