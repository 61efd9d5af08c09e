"""Benchmark: SST block decode + re-encode, device-resident (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W --blocks B]

One "step" = one fused decode -> re-encode pass (sstc_roundtrip_blocks) over
B blocks resident in HBM (default B = 65 536 uniform 4188 B blocks, 16 B keys /
100 B values = BASELINE config 2).  With --gpus N > 1 the script launches N
ranks itself (torch.distributed.run as a child process, before any GPU call;
under an external torchrun it joins as one rank), rank r on GPU r; every rank
owns its own disjoint shard of B blocks (weak scaling, no data-path
collective); the barrier and the per-rank timings (gathered over RCCL) are the
only communication.  value = input bytes of all ranks / max-over-ranks time,
GiB/s; per_rank lists each GPU's GiB/s and roofline fraction.

Input blocks are produced on the GPU by the codec's own encoder from records
generated on the host (synthetic, deterministic); a warm-up round trip is
checked for identity before timing.

roofline: the dominant (only) kernel of a step is rt_kernel.  Algorithmic bytes per launch
= B x (4188 read + 4188 written); duration = span of HIP
events on the codec's stream at the two ends of the K timed calls / K
(includes the launch gaps between back-to-back calls, so the fraction is
slightly conservative against the rocprofv3 kernel average); peak = 8 TB/s (MI355X_MICROARCH.md).
traffic = HBM bytes per launch from rocprofv3 PMC passes (FETCH_SIZE x 2 for
gfx950 + WRITE_SIZE, KB units), read from profiles/pmc_traffic.json when it was
collected for this workload, else null.

cpu_baseline: the reference's own code (oracle/_ref/libsstref.so: BlockReader +
BlockReaderIterator -> BlockBuilder), one thread, on a bounded sample of the
same blocks, pinned to one CPU; falls back to the clean-room oracle ("port")
if the reference build is absent.  cpu_baseline_all: the same on nproc host
threads (the job's CPU share), each pinned to its own CPU; generous, the
reference compacts on one thread.

legs (N=1): decode alone and encode alone over the same blocks, each with its
own roofline sub-object; compact = BASELINE config 3 (8 SSTs x 1 M records)
through the device compaction job sstc_compact, verified against the
reference's output hashes, with its own roofline; compact.files = the same job
file -> file (sstc_compact_files, fsync on) with the reference's own loop on
the same files beside it as compact.cpu_baseline (like for like).
legs.compact_config4 (every N): BASELINE config 4 -- each rank compacts its own
128-SST shard (workload.config_inputs(4, rank)) with one sstc_compact job,
verified against the reference's outputs for that shard; per-rank GiB/s and
roofline fraction, aggregate = all ranks' input bytes / max-over-ranks time.

Input pin: the GPU-built block buffer is hashed and must equal the reference
BlockBuilder's encoding of the same records (tests/golden/bench_inputs.json).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))

import sstcodec  # noqa: E402
from sstcodec import launch  # noqa: E402
from sstcodec import shard  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec.codec import RecordTable  # noqa: E402
from sstcodec._lib import check  # noqa: E402

PER_BLOCK = 28
BLOCK_BYTES = 4188
HBM_PEAK_GBPS = 8000.0
METRIC = "GiB/s SST block decode+re-encode (device-resident), 4 KiB blocks, 1/2/4/8 GPU"


def make_blocks(codec, dev, nblocks, rank):
    """Uniform blocks for this rank's shard: keys k%015d of global record
    index, 100 B values from splitmix64 (seed 1 + rank), ascending txns."""
    n = nblocks * PER_BLOCK
    start, end = shard.record_range(rank, n)
    rec = W.uniform_records(n, key_index=np.arange(start, end, dtype=np.uint64), seed=1 + rank,
                            txn_start=1 + start)
    table = RecordTable.from_numpy(rec, dev)
    first = torch.arange(0, n + 1, PER_BLOCK, dtype=torch.int64, device=dev)
    ksrc = torch.from_numpy(rec["key_src"]).to(dev)
    vsrc = torch.from_numpy(rec["val_src"]).to(dev)
    src, off, ln = codec.encode(table, ksrc, vsrc, first)
    del table, ksrc, vsrc
    return src, off[:-1].contiguous(), ln.contiguous()


def input_pin(src, nblocks, rank):
    """SHA-256 of the GPU-built input buffer against the reference BlockBuilder's
    encoding of the same records (tests/golden/bench_inputs.json, made by
    tests/golden/make_golden_bench.py from /root/reference/sstable/block_builder.cc).
    Returns True / False, or None when no fixture covers (rank, nblocks)."""
    import hashlib
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_inputs.json")) as f:
            cases = json.load(f)["cases"]
    except (OSError, ValueError, KeyError):
        return None
    want = [c["sha256"] for c in cases if c["rank"] == rank and c["blocks"] == nblocks]
    if not want:
        return None
    h = hashlib.sha256()
    step = 64 << 20
    for lo in range(0, src.numel(), step):
        h.update(src[lo:lo + step].cpu().numpy().tobytes())
    return h.hexdigest() == want[0]


def time_roundtrip(codec, src, dst, off, ln, steps, warmup, stream, ranks):
    import ctypes
    nb = off.numel()
    out_len = torch.empty(nb, dtype=torch.int64, device=src.device)
    status = torch.empty(nb, dtype=torch.int32, device=src.device)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    args = (ptr(src), ptr(dst), ptr(off), ptr(ln), nb, 0, ptr(out_len), ptr(status))
    codec._stream()
    for _ in range(warmup):
        rc = codec.roundtrip_raw(*args)
        assert rc == 0
    # HIP events at the two ends of the timed region only: an event recorded
    # between launches adds ~2.5 us per step (tools/ab_launch.py,
    # profiles/r01_ab_launch.log); the per-launch average is their span / K
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ranks.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        codec.roundtrip_raw(*args)
    e1.record(stream)
    torch.cuda.synchronize()
    ranks.barrier()
    wall = time.perf_counter() - t0
    per_launch = [e0.elapsed_time(e1) / steps] * steps
    return wall, per_launch, out_len, status


def cpu_baseline(sample_src, sample_off, sample_len, seconds=10.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    kind = "reference"
    try:
        lib = O.RefLib()
        run = lambda: lib.roundtrip(sample_src, sample_off, sample_len, dst=dst)  # noqa: E731
    except (FileNotFoundError, OSError):
        kind = "port"
        lib = O.Oracle()
        run = lambda: lib.roundtrip(sample_src, sample_off, sample_len, 0)  # noqa: E731
    dst = np.zeros_like(sample_src)
    old = os.sched_getaffinity(0)
    cpu = current_cpu()
    os.sched_setaffinity(0, {cpu})
    run()  # warm
    passes = 0
    t0 = time.perf_counter()
    while True:
        run()
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    os.sched_setaffinity(0, old)
    nbytes = passes * int(sample_len.sum())
    return {"value": nbytes / el / 2 ** 30, "unit": "GiB/s", "cores": 1, "kind": kind, "pinned_cpu": cpu,
            "sample": f"{sample_len.size} blocks x {int(sample_len[0])} B (same uniform workload), "
                      f"{passes} passes in {el:.1f} s, 1 thread, decode (BlockReader/Iterator) + "
                      f"re-encode (BlockBuilder) in host memory"}


def cpu_baseline_threads(sample_src, sample_off, sample_len, threads, seconds=5.0):
    """The same reference round trip on `threads` host threads (= nproc, the CPU
    share this job is given), blocks split into contiguous ranges, thread k
    pinned to the k-th CPU of the affinity mask (ctypes releases the GIL).  A
    GENEROUS baseline: the reference runs one compaction at a time on one
    thread (db/db_impl.cc:548)."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    try:
        lib = O.RefLib()
    except (FileNotFoundError, OSError):
        return None
    cpus = sorted(os.sched_getaffinity(0))
    n_aff = len(cpus)
    threads = max(1, min(threads, n_aff))
    c0 = cpus.index(current_cpu()) if current_cpu() in cpus else 0
    cpus = (cpus[c0:] + cpus[:c0])[:threads]
    nb = sample_off.size
    parts = np.array_split(np.arange(nb), threads)
    dsts = [np.zeros_like(sample_src) for _ in range(threads)]
    done = [0] * threads
    stop = time.perf_counter() + seconds

    def work(k):
        os.sched_setaffinity(0, {cpus[k]})  # pid 0 = this thread (Linux)
        idx = parts[k]
        o, ln = sample_off[idx], sample_len[idx]
        while time.perf_counter() < stop:
            lib.roundtrip(sample_src, o, ln, dst=dsts[k])
            done[k] += int(ln.sum())

    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    return {"value": sum(done) / el / 2 ** 30, "unit": "GiB/s", "cores": threads, "kind": "reference",
            "nproc": nproc(), "os_cpu_count": os.cpu_count(), "affinity_cpus": n_aff,
            "pinning": f"thread k -> CPU {cpus[0]}+k of the affinity mask (sched_setaffinity; start = the CPU "
                                 f"the bench ran on)",
            "label": "generous: the reference compacts on one thread",
            "sample": f"{nb} blocks split over {threads} threads, {el:.1f} s"}


def e2e_rate(codec, src, off, ln, chunk_bytes=16 << 20, reps=5):
    """Host-memory -> host-memory rate through the library's own pipeline
    (sstc_roundtrip_host: pinned H2D on an upload stream, rt_kernel on the
    context's stream, D2H on a download stream, 3 device buffer pairs ordered
    by events).  Returns GiB/s of input bytes.  PCIe-bound by construction
    (profiles/r01_pcie_probe.log: 49 GB/s each way when both directions run)."""
    nbytes = src.numel()
    h_src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_src.copy_(src.cpu())
    o = off.cpu().numpy().view(np.uint64)
    n = ln.cpu().numpy().view(np.uint64)
    _, st = codec.roundtrip_host(h_src, h_dst, o, n, chunk_bytes=chunk_bytes)
    ok = bool(torch.equal(h_dst, h_src)) and bool((st == 0).all())
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.roundtrip_host(h_src, h_dst, o, n, chunk_bytes=chunk_bytes)
    el = (time.perf_counter() - t0) / reps
    return {"value": round(nbytes / el / 2 ** 30, 2), "unit": "GiB/s", "verified": ok,
            "how": f"sstc_roundtrip_host: pinned host -> H2D -> rt_kernel -> D2H -> pinned host, "
                   f"{chunk_bytes >> 20} MiB chunks, upload / kernel / download streams, 3 device buffer pairs, "
                   f"{nbytes} B input"}


def e2e_files(codec, src, off, ln, chunk_blocks=8192, reps=3, io_threads=4):
    """SURVEY.md §8(d) end-to-end: the config-2 blocks as one file in the
    page cache -> pread into pinned memory -> sstc_roundtrip_host (H2D, the
    fused kernel, D2H) -> pwrite, by chunks of `chunk_blocks` blocks (32 MiB)
    with the reads, the codec and the writes of consecutive chunks overlapped
    (a reader and a writer stage, each chunk's pread / pwrite split over
    io_threads threads; three pinned buffer pairs).
    No fsync (the reference's fsync is a disk property, not the codec's);
    returns GiB/s of input bytes and the serial read / codec / write times."""
    import concurrent.futures as cf
    import tempfile
    nb = off.numel()
    o = off.cpu().numpy().view(np.uint64).astype(np.int64)
    n = ln.cpu().numpy().view(np.uint64).astype(np.int64)
    nbytes = int(o[-1] + n[-1])
    chunks = [(b0, min(nb, b0 + chunk_blocks)) for b0 in range(0, nb, chunk_blocks)]
    spans = [(int(o[b0]), int(o[b1 - 1] + n[b1 - 1])) for b0, b1 in chunks]
    cap = max(hi - lo for lo, hi in spans)
    nbuf = 3
    h_in = [torch.empty(cap, dtype=torch.uint8, pin_memory=True) for _ in range(nbuf)]
    h_out = [torch.empty(cap, dtype=torch.uint8, pin_memory=True) for _ in range(nbuf)]
    rel = [((o[b0:b1] - lo).astype(np.uint64), n[b0:b1].astype(np.uint64)) for (b0, b1), (lo, _) in zip(chunks, spans)]
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        pin, pout = os.path.join(td, "blocks.in"), os.path.join(td, "blocks.out")
        src.cpu().numpy().tofile(pin)
        fi = os.open(pin, os.O_RDONLY)
        fo = os.open(pout, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        os.ftruncate(fo, nbytes)

        io_pool = cf.ThreadPoolExecutor(2 * io_threads)

        def part(i, k):  # k-th of io_threads slices of chunk i
            lo, hi = spans[i]
            step = (hi - lo + io_threads - 1) // io_threads
            return min(hi - lo, k * step), min(hi - lo, (k + 1) * step)

        def rd_part(i, k):
            a, b = part(i, k)
            mv = memoryview(h_in[i % nbuf].numpy())[a:b]
            got = 0
            while got < b - a:
                got += os.preadv(fi, [mv[got:]], spans[i][0] + a + got)

        def wr_part(i, k):
            a, b = part(i, k)
            mv = memoryview(h_out[i % nbuf].numpy())[a:b]
            put = 0
            while put < b - a:
                put += os.pwrite(fo, mv[put:], spans[i][0] + a + put)

        def rd(i):  # the chunk's slices read in parallel (page-cache copies scale with threads)
            for f in [io_pool.submit(rd_part, i, k) for k in range(io_threads)]:
                f.result()

        def wr(i):
            for f in [io_pool.submit(wr_part, i, k) for k in range(io_threads)]:
                f.result()

        def one_pass():
            with cf.ThreadPoolExecutor(1) as rpool, cf.ThreadPoolExecutor(1) as wpool:
                reads = {0: rpool.submit(rd, 0)}
                writes = {}
                for i in range(len(chunks)):
                    reads.pop(i).result()
                    if i + 1 < len(chunks):
                        if i + 1 - nbuf in writes:
                            writes.pop(i + 1 - nbuf).result()  # its output buffer is reused by chunk i + 1
                        reads[i + 1] = rpool.submit(rd, i + 1)
                    if i - nbuf in writes:
                        writes.pop(i - nbuf).result()
                    _, st = codec.roundtrip_host(h_in[i % nbuf], h_out[i % nbuf], rel[i][0], rel[i][1])
                    assert (st == 0).all()
                    writes[i] = wpool.submit(wr, i)
                for f in writes.values():
                    f.result()

        one_pass()  # warm: page cache, pinned buffers, the codec's pipe
        t0 = time.perf_counter()
        for _ in range(reps):
            one_pass()
        el = (time.perf_counter() - t0) / reps
        ok = bool(np.array_equal(np.fromfile(pout, np.uint8), src.cpu().numpy()[:nbytes]))
        # the stages one at a time (what the overlap hides)
        t0 = time.perf_counter()
        for i in range(len(chunks)):
            rd(i)
        t_rd = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i in range(len(chunks)):
            codec.roundtrip_host(h_in[i % nbuf], h_out[i % nbuf], rel[i][0], rel[i][1])
        t_cd = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i in range(len(chunks)):
            wr(i)
        t_wr = time.perf_counter() - t0
        io_pool.shutdown()
        os.close(fi)
        os.close(fo)
    return {"value": round(nbytes / el / 2 ** 30, 2), "unit": "GiB/s", "verified": ok, "io_threads": io_threads,
            "serial_s": {"pread": round(t_rd, 4), "codec_host_to_host": round(t_cd, 4), "pwrite": round(t_wr, 4)},
            "how": f"page-cache file -> pread -> pinned -> sstc_roundtrip_host -> pinned -> pwrite (no fsync), "
                   f"{len(chunks)} chunks of {chunk_blocks} blocks, reads / codec / writes of consecutive chunks "
                   f"overlapped, {io_threads} threads per pread / pwrite, {nbytes} B input"}


def hbm_variant(codec, dev, nblocks, steps=10):
    """The same fused round trip over nblocks (default 4 x config 2, ~1.1 GB in
    + 1.1 GB out: beyond the 256 MiB Infinity Cache, so HBM-bound).  HIP-event
    span of `steps` back-to-back launches / steps; identity checked."""
    import ctypes
    src, off, ln = make_blocks(codec, dev, nblocks, 0)
    pinned = input_pin(src, nblocks, 0)
    if pinned is False:
        raise SystemExit("1 GiB variant: GPU-built blocks differ from the reference BlockBuilder's")
    dst = torch.empty_like(src)
    out_len = torch.empty(nblocks, dtype=torch.int64, device=dev)
    status = torch.empty(nblocks, dtype=torch.int32, device=dev)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    args = (ptr(src), ptr(dst), ptr(off), ptr(ln), nblocks, 0, ptr(out_len), ptr(status))
    codec._stream()
    stream = torch.cuda.current_stream(dev)
    for _ in range(2):
        assert codec.roundtrip_raw(*args) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        codec.roundtrip_raw(*args)
    e1.record(stream)
    torch.cuda.synchronize()
    ok = bool(torch.equal(dst, src)) and bool((status == 0).all())
    ms = e0.elapsed_time(e1) / steps
    alg = 2 * nblocks * BLOCK_BYTES
    achieved = alg / (ms * 1e-3) / 1e9
    del src, dst, off, ln, out_len, status
    torch.cuda.empty_cache()
    cp = copy_peak(codec, dev, (alg // 2 + 15) // 16 * 16)
    return {"copy_peak_GBps": round(cp, 1), "frac_of_copy_peak": round(achieved / cp, 4), "blocks": nblocks, "input_bytes": nblocks * BLOCK_BYTES, "launch_ms_events": round(ms, 5),
            "GiBps_in": round(nblocks * BLOCK_BYTES / (ms * 1e-3) / 2 ** 30, 1), "achieved_GBps": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "verified": ok, "input_sha256_equals_reference": pinned,
            "why": "4x config 2 so the working set exceeds the 256 MiB Infinity Cache (HBM-bound)"}


def read_traffic(nblocks):
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if int(d.get("nblocks", -1)) == nblocks and d.get("kernel") and d.get("hbm_bytes_per_launch"):
            return float(d["hbm_bytes_per_launch"])
    except (OSError, ValueError):
        pass
    return None


def copy_peak(codec, dev, nbytes, reps=10):
    """Copy ceiling of the box: sstc_copy_probe (plain 16 B non-temporal copy
    kernel of the library) over nbytes, HIP events on the codec's stream.
    Returns read+written GB/s."""
    import ctypes
    a = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    codec._stream()
    stream = torch.cuda.current_stream(dev)
    run = lambda: check(codec.lib.sstc_copy_probe(codec.h, ctypes.c_void_p(a.data_ptr()),  # noqa: E731
                                                  ctypes.c_void_p(b.data_ptr()), nbytes), "sstc_copy_probe")
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2 * nbytes / (ms * 1e-3) / 1e9


def nproc():
    """GNU nproc (honours the affinity mask and OMP_NUM_THREADS, i.e. the
    CPU share a job is given on the GPU box) with os.cpu_count() beside it."""
    import shutil
    import subprocess
    try:
        return int(subprocess.run([shutil.which("nproc") or "nproc"], capture_output=True, text=True,
                                  check=True).stdout.strip())
    except (OSError, ValueError, subprocess.CalledProcessError):
        return len(os.sched_getaffinity(0))


def current_cpu():
    """CPU this thread runs on now (/proc/self/stat field 39): the pinned
    baselines start there rather than at CPU 0, which on a shared host is the
    likeliest to be busy."""
    try:
        with open("/proc/thread-self/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[36])
    except (OSError, ValueError, IndexError):
        return min(os.sched_getaffinity(0))


def time_leg(codec, stream, call, steps, warmup=3):
    """HIP-event span of `steps` back-to-back calls on the codec's stream / steps (ms)."""
    for _ in range(warmup):
        rc = call()
        assert rc == 0, rc
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        call()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def codec_legs(codec, dev, stream, src, off, ln, steps):
    """Decode alone (sstc_decode_blocks: blocks -> SoA record table) and encode
    alone (sstc_encode_blocks: SoA + key/value arenas -> blocks) over the same
    config-2 blocks, each with its own roofline (a decode
    counts B_in + SoA bytes out; an encode counts block bytes out + key/value
    bytes read + SoA bytes read).  Both outputs are verified."""
    import ctypes
    nb = off.numel()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rec_base = codec.count(src, off, ln)
    table, _, status = codec.decode(src, off, ln, rec_base=rec_base)
    nrec = table.n
    c = table.c()
    dec = lambda: codec.lib.sstc_decode_blocks(codec.h, P(src), P(off), P(ln), nb, P(rec_base), c,  # noqa: E731
                                               sstcodec.SSTC_TXN_COMPAT, P(status))
    codec._stream()
    dms = time_leg(codec, stream, dec, steps)
    ok_dec = bool((status == 0).all()) and nrec == nb * PER_BLOCK
    soa = 33 * nrec
    d_alg = nb * BLOCK_BYTES + soa
    # encode from the decoded table: keys / values are read in place from the
    # input blocks (key_off / val_off point into src), first = every 28 records
    first = torch.arange(0, nrec + 1, PER_BLOCK, dtype=torch.int64, device=dev)
    dst = torch.zeros_like(src)
    out_off = torch.empty(nb + 1, dtype=torch.int64, device=dev)
    out_len = torch.empty(nb, dtype=torch.int64, device=dev)
    enc = lambda: codec.lib.sstc_encode_blocks(codec.h, P(src), P(src), c, nrec, P(first), nb, 0,  # noqa: E731
                                               P(dst), P(out_off), P(out_len))
    ems = time_leg(codec, stream, enc, steps)
    ok_enc = bool(torch.equal(dst, src))
    kv = nrec * (16 + 100)
    e_alg = nb * BLOCK_BYTES + kv + soa
    leg = lambda ms, alg, kern, how, ok: {  # noqa: E731
        "ms": round(ms, 5), "GiBps_blocks": round(nb * BLOCK_BYTES / (ms * 1e-3) / 2 ** 30, 1),
        "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "alg_bytes_per_launch": alg, "kernel": kern, "bytes": how},
        "verified": ok}
    return {"decode": leg(dms, d_alg, "decode_kernel", f"{nb} x {BLOCK_BYTES} B blocks read + {nrec} x 33 B SoA "
                          "records written", ok_dec),
            "encode": leg(ems, e_alg, "enc_offsets_kernel (block lengths + offsets, one kernel) + enc_lds_kernel<0> (entry offsets scanned in the block wave; blocks past an LDS slot by their own wave)",
                          f"{nb} x {BLOCK_BYTES} B blocks written + {nrec} x 116 B key/value read + "
                          f"{nrec} x 33 B SoA read", ok_enc)}


def read_compact_traffic(workload):
    """HBM bytes per sstc_compact call from the PMC passes of
    tools/pmc_compact_job.sh (profiles/pmc_compact*.json), or None."""
    for name in ("pmc_compact.json", "pmc_compact_c4.json", "pmc_compact_c5.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
            if d.get("workload") == workload:
                return float(d["hbm_bytes_per_call"])
        except (OSError, ValueError, KeyError):
            pass
    return None


def _sha(b):
    import hashlib
    return hashlib.sha256(b).hexdigest()


class GpuCompaction:
    """One compaction job (db/compact.cc:232-322) on this rank's GPU: the input
    SSTs are written by the flush-path sstc::TableBuilder into `td` (and must
    hash to the reference TableBuilder's files, when a fixture covers them),
    uploaded once, indexed on the device (sstc_open_tables); run() is one
    device-resident sstc_compact call; outputs() hashes every output SST."""

    def __init__(self, codec, dev, stream, td, record_sets, fixture, block_threshold=4096, table_limit=32 << 20):
        import ctypes
        from sstcodec._lib import CompactParams, CompactResult
        from sstcodec.table import build_table
        self.codec, self.dev, self.stream = codec, dev, stream
        files, self.paths = [], []
        self.inputs_ok = None if fixture is None else True
        for i, rec in enumerate(record_sets):
            p = os.path.join(td, f"in{i}.sst")
            fs, _ = build_table(codec, p, rec, block_threshold)
            img = np.fromfile(p, np.uint8)
            if fixture is not None:
                w = fixture["inputs"][i]
                self.inputs_ok &= fs == w["file_size"] and _sha(img.tobytes()) == w["sha256"]
            files.append(img)
            self.paths.append((p, fs))
        if self.inputs_ok is False:
            raise SystemExit("compaction leg: input SSTs differ from the reference TableBuilder's")
        self.src = torch.from_numpy(np.concatenate(files)).to(dev)
        sizes = [f.size for f in files]
        del files
        idx = codec.open_tables(self.src, sizes, strict=True)
        self.bo, self.bl, self.h_tfb = idx["blk_off"], idx["blk_len"], idx["table_first_block"]
        self.cap = int(self.src.numel()) + (1 << 20)
        self.dst = torch.empty(self.cap, dtype=torch.uint8, device=dev)
        self.max_t = 1 << 12
        self.toff = torch.zeros(self.max_t + 1, dtype=torch.int64, device=dev)
        self.tlen = torch.zeros(self.max_t, dtype=torch.int64, device=dev)
        self.prm = CompactParams(block_threshold, table_limit, 1, 0)
        self.res = CompactResult()
        self.ntables = len(sizes)
        self.in_bytes = int(self.src.numel())
        self._ct = ctypes

    def run(self):
        ct, P = self._ct, lambda t: self._ct.c_void_p(t.data_ptr())  # noqa: E731
        self.codec._stream()
        check(self.codec.lib.sstc_compact(self.codec.h, P(self.src), P(self.bo), P(self.bl), int(self.bo.numel()),
                                          self.h_tfb.ctypes.data_as(ct.c_void_p), self.ntables,
                                          ct.byref(self.prm), P(self.dst), self.cap, P(self.toff), P(self.tlen),
                                          self.max_t, ct.byref(self.res)), "sstc_compact")

    def sync(self):
        if self.dev.type == "cuda":  # (a host device only in the CPU test of this rank path)
            torch.cuda.synchronize(self.dev)

    def outputs(self):
        """[(sha256, GetFileSize())] of the last call's output SSTs, output bytes."""
        nt = self.res.tables_out
        o = self.toff[: nt + 1].cpu().numpy()
        d = self.dst[: int(o[nt])].cpu().numpy()
        return [(_sha(d[int(o[t]):int(o[t + 1])].tobytes()), int(o[t + 1] - o[t]) + 1) for t in range(nt)], int(o[nt])

    def free(self):
        del self.src, self.dst
        if self.dev.type == "cuda":
            torch.cuda.empty_cache()


def time_job(job, steps, ranks=None, warmup=2):
    """K back-to-back calls bracketed by a barrier + device sync on both sides
    (max over ranks is taken by the caller); also the median of `steps` single
    calls (each bracketed by syncs; the job makes host fetches inside)."""
    for _ in range(warmup):
        job.run()
    job.sync()
    singles = []
    for _ in range(steps):
        job.sync()
        t0 = time.perf_counter()
        job.run()
        job.sync()
        singles.append(time.perf_counter() - t0)
    if ranks is not None:
        ranks.barrier()
    job.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        job.run()
    job.sync()
    if ranks is not None:
        ranks.barrier()
    return time.perf_counter() - t0, float(np.median(singles))


def ref_compact_baseline(paths, td, in_bytes, block_threshold=4096, table_limit=32 << 20):
    """The reference's own MergeIterator + TableReaderIterator + TableBuilder
    under the DoCompactJob loop (oracle/_ref/ref_compact, built from
    /root/reference by oracle/Makefile), one pinned thread, on the same input
    files (page-cache-hot), outputs written + fsync'd by the reference's
    TableBuilder (table_builder.cc:147-177)."""
    import subprocess
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_compact")
    if not os.path.exists(ref):
        return None
    od = os.path.join(td, "ref_out")
    os.makedirs(od, exist_ok=True)
    cpu = current_cpu()
    t0 = time.perf_counter()
    r = subprocess.run([ref, od, str(block_threshold), str(table_limit), "1"] +
                       [x for p, fs in paths for x in (p, str(fs))],
                       capture_output=True, text=True, preexec_fn=lambda: os.sched_setaffinity(0, {cpu}))
    el = time.perf_counter() - t0
    if r.returncode != 0:
        return None
    return {"value": round(in_bytes / el / 2 ** 30, 3), "unit": "GiB/s", "seconds": round(el, 3), "cores": 1,
            "kind": "reference", "pinned_cpu": cpu,
            "sample": "the whole job once: the reference's MergeIterator + TableReaderIterator + TableBuilder under "
                      "the DoCompactJob loop (oracle/_ref/ref_compact), input files page-cache-hot, outputs written + "
                      "fsync'd like the reference"}


def files_leg(codec, paths, td, fixture, in_bytes, reps=3, io_threads=8):
    """The path north_star names end to end (SST files -> SST files):
    sstc_compact_files over the input files -- host-side index parse, chunked
    preads into pinned memory overlapped with H2D, the device job, D2H + one
    pwrite + fsync per output SST (io/linux_file.cc:138-195,
    table_builder.cc:147-177) -- fsync ON, like the reference's TableBuilder.
    Median of `reps` runs; every output verified against the reference's hashes."""
    od = os.path.join(td, "files_out")
    os.makedirs(od, exist_ok=True)
    pipe = sstcodec.FilePipe(codec, io_threads=io_threads)
    ps, sz = [p for p, _ in paths], [fs for _, fs in paths]
    runs = []
    ok = True
    for _ in range(reps + 1):
        for f in os.listdir(od):  # fresh outputs each run (the job opens existing files without O_TRUNC)
            os.unlink(os.path.join(od, f))
        outs, tm = pipe.compact_files(ps, sz, od + "/", 0, fixture["block_threshold"], fixture["table_limit"], 1,
                                      fsync=True)
        runs.append(tm)
        if fixture is not None:
            got = []
            for sid, fsize, _, _ in outs:
                with open(os.path.join(od, f"{sid}.sst"), "rb") as f:
                    got.append((_sha(f.read()), fsize))
            ok &= got == [(w["sha256"], w["file_size"]) for w in fixture["outputs_base1"]]
    pipe.close()
    runs = runs[1:]  # the first run warms the pipe's pinned staging
    k = int(np.argsort([r["total_s"] for r in runs])[len(runs) // 2])
    t = runs[k]
    return {"what": f"sstc_compact_files: {len(ps)} SST files -> {len(outs)} SST files, fsync on, {io_threads} I/O "
                    f"threads, median of {reps}",
            "s_median": round(t["total_s"], 4), "GiBps_in": round(in_bytes / t["total_s"] / 2 ** 30, 2),
            "breakdown_s": {k2: round(v, 4) for k2, v in t.items() if k2 != "total_s"},
            "verified_vs_reference": bool(ok)}


COMPACT_WORKLOADS = {
    3: "config3: 8 SSTs x 1 M records (16 B keys, 100 B values) -> 28 SSTs, sstc_compact, device-resident",
    5: "config5: 8 SSTs x 5000 records over a shared 20 000-key space (Zipf 8 B - 64 KiB values, 10 % DELETE, "
       "overlapping keys: the drop / overwrite path) -> 14 SSTs, sstc_compact, device-resident",
}


def compact_leg(codec, dev, stream, steps, cpu_ref=True, files=True, config=3, dropin=True):
    """BASELINE config 3 (or 5) -- the compaction hot path north_star replaces
    (db/compact.cc:232-322): config 3 = 8 SSTs x 1 M records (16 B keys, 100 B
    values, disjoint interleave) -> 28 output SSTs; config 5 = Zipf values
    8 B - 64 KiB with overlapping keys and DELETEs -> 14 SSTs.  sstc_compact
    (decode, k-way merge, keep/drop, 32 MiB table split, 4 KiB block split,
    encode, meta, footers).  Inputs are written by the flush-path
    sstc::TableBuilder and must hash to the reference TableBuilder's files;
    every output must hash to the reference's compaction
    (tests/golden/compaction_configs.json).  Device-resident time = median of
    `steps` calls, each bracketed by device syncs.  Roofline: the job must
    read every input byte once and write every output byte once: algorithmic
    bytes = input + output bytes.  `files`: the same job file -> file
    (sstc_compact_files, fsync on) beside the reference's own loop on the
    same files (cpu_baseline, like for like).  `dropin`: PickCompact under the
    UNCHANGED db/compact.cc with the drop-ins (dropin_leg)."""
    import shutil
    import tempfile
    tag = f"config{config}"
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "compaction_configs.json")))[tag]
    td = tempfile.mkdtemp(prefix=f"sstc_bench_c{config}_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        sets = W.config_inputs(config)
        ranges = [record_key_range(r) for r in sets]
        job = GpuCompaction(codec, dev, stream, td, sets, fx)
        del sets
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        _, t = time_job(job, steps)
        e0.record(stream)
        job.run()
        e1.record(stream)
        torch.cuda.synchronize()
        got, out_bytes = job.outputs()
        ok = got == [(w["sha256"], w["file_size"]) for w in fx["outputs_base1"]]
        in_bytes, res = job.in_bytes, job.res
        paths = job.paths
        job.free()
        alg = in_bytes + out_bytes
        leg = {"workload": COMPACT_WORKLOADS[config], "steps": steps, "ms_median": round(t * 1e3, 4),
               "ms_events_one_call": round(e0.elapsed_time(e1), 4),
               "GiBps_in": round(in_bytes / t / 2 ** 30, 1), "records_in": res.records_in,
               "records_kept": res.records_kept, "tables_out": res.tables_out, "input_bytes": in_bytes,
               "output_bytes": out_bytes, "verified_vs_reference": ok, "inputs_equal_reference": job.inputs_ok,
               "roofline": {"bound": "hbm", "achieved": round(alg / t / 1e9, 1), "peak": HBM_PEAK_GBPS,
                            "unit": "GB/s", "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4),
                            "traffic": read_compact_traffic(tag), "alg_bytes_per_call": alg,
                            "alg": "input bytes read once + output bytes written once (a copy's traffic)",
                            "kernel": "sstc_compact (whole job, ~30 kernels; wall time incl. its host syncs)"}}
        if not ok:
            raise SystemExit(f"{tag} compact leg: outputs differ from the reference's compaction: timing invalid")
        if files:
            leg["files"] = files_leg(codec, paths, td, fx, in_bytes)
        if cpu_ref:
            base = ref_compact_baseline(paths, td, in_bytes)
            if base:
                base["compare_with"] = "legs.*.files (file -> file, fsync on): the like-for-like GPU number"
                leg["cpu_baseline"] = base
        if dropin:
            leg["dropin"] = dropin_leg(paths, ranges, fx, td, in_bytes)
        return leg
    finally:
        shutil.rmtree(td, ignore_errors=True)


def record_key_range(rec):
    """first and last key of a record set (what VersionEdit records for an input SST)"""
    ko, kl, ks = rec["key_off"], rec["key_len"], rec["key_src"]
    return (bytes(ks[int(ko[0]):int(ko[0]) + int(kl[0])]), bytes(ks[int(ko[-1]):int(ko[-1]) + int(kl[-1])]))


def dropin_leg(paths, ranges, fixture, td, in_bytes, reps=2):
    """Compact::PickCompact -> DoCompactJob, the reference's
    own db/compact.cc compiled UNCHANGED with include/dropin/ first on the
    include path (oracle/Makefile target `dropin`: the engine build, linked
    with libsstcodec.so), so its MergeIterator merges on the device
    (include/dropin/db/merge_iterator.h: inputs mapped + uploaded once,
    sstc_merge_records), its TableReaderIterators are the drop-in readers and
    every output SST is built by sstc::TableBuilder (device encode from the
    resident inputs, O_DIRECT write + fsync); timed beside the reference AS
    WRITTEN (oracle/_ref/ref_pick_compact: the same compact.cc with the
    reference's merge_iterator.cc, table_reader_iterator.cc and
    table_builder.cc) on the same input files, same host, one process each,
    dirty pages synced before every run.  The drop-in's outputs are verified
    against the reference's fixed-semantics outputs; seconds = PickCompact
    wall time as the harness prints it (codec context opened before the timer,
    as an engine does at DB open)."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "compact_dropin")
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_pick_compact")
    if not os.path.exists(exe):
        return None
    args = [str(fixture["block_threshold"]), str(fixture["table_limit"])]
    for (p, fs), (lo, hi) in zip(paths, ranges):
        args += [p, str(fs), lo.hex() or "-", hi.hex() or "-"]

    def run(binary, tag, i, env=None):
        d = os.path.join(td, f"pick_{tag}_{i}")
        os.makedirs(d)
        os.sync()
        r = subprocess.run([binary, d] + args, capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, **(env or {})))
        if r.returncode != 0:
            raise SystemExit(f"dropin leg: {tag} failed: {r.stderr[-500:]}")
        t = float(next(ln.split()[1] for ln in r.stdout.splitlines() if ln.startswith("time ")))
        outs = [ln.split() for ln in r.stdout.splitlines() if ln.startswith("out ")]
        return t, outs, d

    gpu, cpu, ok = [], [], True
    for i in range(reps):
        t, outs, d = run(exe, "dropin", i)
        got = []
        for o in outs:
            with open(o[1], "rb") as f:
                got.append((_sha(f.read()), int(o[2])))
        ok &= got == [(w["sha256"], w["file_size"]) for w in fixture["outputs_base1"]]
        gpu.append(t)
        import shutil
        shutil.rmtree(d, ignore_errors=True)
        if os.path.exists(ref):  # (config 5 as written needs its freed blocks kept mapped, else it crashes)
            tr, _, d = run(ref, "ref", i, {"GLIBC_TUNABLES": "glibc.malloc.trim_threshold=17179869184"})
            cpu.append(tr)
            shutil.rmtree(d, ignore_errors=True)
    if not ok:
        raise SystemExit("dropin leg: the unchanged compact.cc with the drop-ins wrote other bytes than the reference")
    # one more run with the library's host trace on (SSTC_TRACE_HOST=1): where the seconds go
    phases = None
    try:
        d = os.path.join(td, "pick_traced")
        os.makedirs(d)
        os.sync()
        r = subprocess.run([exe, d] + args, capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, SSTC_TRACE_HOST="1"))
        import re
        import shutil
        shutil.rmtree(d, ignore_errors=True)
        tot = {}
        for ln in r.stderr.splitlines():
            m = re.match(r"\[sstc\] (resident inputs: .*?|MergeIterator life.*?) ([0-9.]+) ms$", ln)
            if m:
                tot[m.group(1)] = tot.get(m.group(1), 0.0) + float(m.group(2))
            elif ln.startswith("[sstc] Finish"):
                tot["Finish (sum)"] = tot.get("Finish (sum)", 0.0) + float(ln.split(": ")[1].split(" ms")[0])
                tot["Finish calls"] = tot.get("Finish calls", 0) + 1
                for part, v in re.findall(r"(pwrite|fsync) ([0-9.]+)", ln):
                    tot[f"Finish {part} (sum)"] = tot.get(f"Finish {part} (sum)", 0.0) + float(v)
        if r.returncode == 0 and tot:
            t = float(next(ln.split()[1] for ln in r.stdout.splitlines() if ln.startswith("time ")))
            phases = {"s": round(t, 4), **{k: round(v, 2) for k, v in tot.items()}}
    except (OSError, ValueError, StopIteration, subprocess.TimeoutExpired):
        phases = None
    g = float(np.median(gpu))
    leg = {"what": "Compact::PickCompact (db/compact.cc unchanged) with the drop-in MergeIterator (device merge), "
                   "TableReaderIterator and TableBuilder (device encode), input files page-cache-hot, outputs "
                   "written + fsync'd", "s_runs": [round(x, 4) for x in gpu], "s_median": round(g, 4),
           "GiBps_in": round(in_bytes / g / 2 ** 30, 3), "verified_vs_reference": bool(ok)}
    if phases:
        leg["phases_ms_traced_run"] = phases
    if cpu:
        c = float(np.median(cpu))
        leg["cpu_baseline"] = {"value": round(c, 4), "unit": "s", "s_runs": [round(x, 4) for x in cpu],
                               "cores": 1, "kind": "reference",
                               "sample": "the same PickCompact with the reference's own merge_iterator.cc, "
                                         "table_reader_iterator.cc and table_builder.cc (oracle/_ref/"
                                         "ref_pick_compact), same input files, same host"}
        leg["ratio_to_reference"] = round(g / c, 3)
    return leg


class HostPlumbing:
    """--plumbing stand-in for GpuCompaction (no GPU): the same shard, rank
    and aggregation path, with a host merge of the shard's key indices as the
    "job".  Not a measurement."""

    def __init__(self, record_sets):
        self.keys = [np.asarray(r["key_src"]).reshape(-1, 16) for r in record_sets]
        self.in_bytes = sum(int(np.asarray(r["key_src"]).size + np.asarray(r["val_src"]).size)
                            for r in record_sets)
        self.inputs_ok = None
        self.out = None

    def run(self):
        allk = np.concatenate(self.keys)
        self.out = allk[np.lexsort(allk.T[::-1])]

    def sync(self):
        pass

    def outputs(self):
        return [(_sha(self.out.tobytes()), self.out.size)], self.in_bytes

    def key_range(self):
        return int(bytes(self.out[0]).decode()[1:]), int(bytes(self.out[-1]).decode()[1:])

    def free(self):
        pass


def config4_leg(ranks, make_job, steps, fixture_of):
    """BASELINE config 4 at N GPUs: 1024 input SSTs sharded 128 per GPU
    (SURVEY.md §8(e)), rank r compacting its own key-range-disjoint shard
    (workload.config_inputs(4, r)) with its own job -- exactly 8 independent
    DoCompactJob runs (db/compact.cc:232-322), no data-path collective.  Each
    rank verifies its outputs against the reference's
    (compaction_configs.json "config4_rank{r}"); value = all ranks' input
    bytes x K / max-over-ranks wall time of K back-to-back calls (barrier +
    device sync on both sides)."""
    job, fixture = make_job(ranks.rank), fixture_of(ranks.rank)
    wall, single = time_job(job, steps, ranks)
    got, out_bytes = job.outputs()
    ok = None if fixture is None else got == [(w["sha256"], w["file_size"]) for w in fixture["outputs_base1"]]
    lo, hi = job.key_range() if hasattr(job, "key_range") else (-1, -1)
    in_bytes = job.in_bytes
    job.free()
    per = ranks.gather([wall, single, in_bytes, out_bytes, -1 if ok is None else int(ok), lo, hi])
    wall_max = max(p[0] for p in per)
    total_in = sum(p[2] for p in per)
    rows = []
    for r, (w, s1, ib, ob, okr, klo, khi) in enumerate(per):
        frac = (ib + ob) / s1 / 1e9 / HBM_PEAK_GBPS
        rows.append({"rank": r, "GiBps": round(ib * steps / w / 2 ** 30, 2), "ms_per_call": round(w / steps * 1e3, 4),
                     "ms_single_median": round(s1 * 1e3, 4), "input_bytes": int(ib), "output_bytes": int(ob),
                     "roofline_frac": round(frac, 4), "verified_vs_reference": None if okr < 0 else bool(okr),
                     "key_index_range": [int(klo), int(khi)] if klo >= 0 else None})
    return {"workload": "config4: 1024 SSTs x 100 k records sharded 128 per GPU, one sstc_compact job per rank "
                        "(device-resident, key-range-disjoint shards)",
            "n_gpus": ranks.world, "steps": steps, "GiBps_aggregate": round(total_in * steps / wall_max / 2 ** 30, 2),
            "ms_per_call_max": round(wall_max / steps * 1e3, 4), "scaling": "weak", "per_rank": rows,
            "roofline_note": "per rank: (input + output bytes) / median single-call time / 8 TB/s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); >1 launches them itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=65536, help="blocks per GPU (config 2: 65536)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->device->host rate")
    ap.add_argument("--no-hbm-variant", action="store_true", help="skip the 4x (1 GiB, HBM-bound) measurement")
    ap.add_argument("--no-legs", action="store_true", help="skip the decode-only / encode-only legs")
    ap.add_argument("--no-compact", action="store_true", help="skip the config-3 compaction leg")
    ap.add_argument("--compact-steps", type=int, default=10)
    ap.add_argument("--no-files-leg", action="store_true", help="skip the config-3 file -> file compaction leg")
    ap.add_argument("--no-compact4", action="store_true", help="skip the config-4 (128 SSTs per GPU) leg")
    ap.add_argument("--no-compact5", action="store_true", help="skip the config-5 (Zipf values) leg")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip PickCompact under the unchanged compact.cc (drop-ins vs the reference as written)")
    ap.add_argument("--c4-steps", type=int, default=5)
    ap.add_argument("--c4-keys", type=int, default=100_000, help="records per SST of the config-4 leg")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU-only launcher check (gloo, host copy as the step): NOT a measurement")
    args = ap.parse_args()

    # N ranks: launch them (child processes, before anything touches the GPU)
    rc = launch.relaunch(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    ranks = launch.init_ranks(args.gpus, "gloo" if args.plumbing else "nccl")
    if args.plumbing:
        return plumbing(args, ranks)
    dev = ranks.device
    rank, world = ranks.rank, ranks.world
    stream = torch.cuda.current_stream(dev)

    codec = sstcodec.Codec(ranks.local)
    nb = args.blocks
    codec.reserve(nb, nb * PER_BLOCK)
    src, off, ln = make_blocks(codec, dev, nb, rank)
    torch.cuda.synchronize()
    assert int(ln.min()) == BLOCK_BYTES == int(ln.max())
    pinned = input_pin(src, nb, rank)
    if pinned is False:
        raise SystemExit("GPU-built input blocks differ from the reference BlockBuilder's: timing invalid")
    dst = torch.empty_like(src)

    wall, per_launch, out_len, status = time_roundtrip(codec, src, dst, off, ln, args.steps, args.warmup,
                                                       stream, ranks)
    # correctness of what was timed: identity round trip, no block errors
    ok = bool(torch.equal(dst, src)) and bool((status == 0).all()) and bool((out_len == BLOCK_BYTES).all())
    if not ok:
        raise SystemExit("round trip output differs from input: timing invalid")

    in_bytes = nb * BLOCK_BYTES
    launch_ms = float(np.mean(per_launch))
    alg = 2 * in_bytes  # read + written per launch
    achieved = alg / (launch_ms * 1e-3) / 1e9
    per_rank = ranks.gather([wall, launch_ms])
    wall_max = max(w for w, _ in per_rank)
    total_in = in_bytes * world * args.steps
    value = total_in / wall_max / 2 ** 30
    ms_step = wall_max / args.steps * 1e3
    traffic = read_traffic(nb)

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform 16 B keys k%015d / 100 B splitmix64 values, blocks built on GPU by "
                    "the codec's encoder; identity round trip verified)",
            "input_sha256_equals_reference_blockbuilder": pinned,
            "config": {"workload": "config2: batch decode+re-encode of 65536 x 4188 B device-resident "
                                   "blocks per GPU (28 PUTs each), fused rt_kernel",
                       "blocks_per_gpu": nb, "block_bytes": BLOCK_BYTES, "records_per_gpu": nb * PER_BLOCK,
                       "txn_mode": "compat", "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": "rt_kernel", "alg_bytes_per_launch": alg,
                         "launch_ms_events": round(launch_ms, 5)},
        }
        if world > 1:
            out["per_rank"] = [{"rank": r, "GiBps": round(in_bytes * args.steps / w / 2 ** 30, 2),
                                "launch_ms_events": round(lm, 5),
                                "roofline_frac": round(alg / (lm * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
                               for r, (w, lm) in enumerate(per_rank)]
        if world == 1:
            cp = copy_peak(codec, dev, (alg // 2 + 15) // 16 * 16)
            out["roofline"]["copy_peak_GBps"] = round(cp, 1)
            out["roofline"]["frac_of_copy_peak"] = round(achieved / cp, 4)
            if not args.no_legs:
                out["legs"] = codec_legs(codec, dev, stream, src, off, ln, max(10, args.steps // 2))
            if not args.no_compact:
                out.setdefault("legs", {})["compact"] = compact_leg(codec, dev, stream, args.compact_steps,
                                                                     not args.no_cpu_baseline, not args.no_files_leg,
                                                                     dropin=not args.no_dropin)
            if not args.no_compact5:
                out.setdefault("legs", {})["compact_config5"] = compact_leg(
                    codec, dev, stream, args.compact_steps, not args.no_cpu_baseline, False, config=5,
                    dropin=not args.no_dropin)
            if not args.no_hbm_variant:
                out["roofline"]["hbm_1gib"] = hbm_variant(codec, dev, 4 * nb)
            if not args.no_e2e:
                out["e2e_pcie"] = e2e_rate(codec, src, off, ln)
                out["e2e_files"] = e2e_files(codec, src, off, ln)
            if not args.no_cpu_baseline:
                k = min(nb, 16384)
                s = src[: k * BLOCK_BYTES].cpu().numpy()
                o = off[:k].cpu().numpy().view(np.uint64)
                l_ = ln[:k].cpu().numpy().view(np.uint64)
                out["cpu_baseline"] = cpu_baseline(s, o, l_, args.cpu_seconds)
                all_cores = cpu_baseline_threads(s, o, l_, nproc(), min(5.0, args.cpu_seconds))
                if all_cores:
                    out["cpu_baseline_all"] = all_cores
    if not args.no_compact4:
        # every rank: its own 128-SST shard of config 4 (collective call: all ranks run it)
        c4 = compact4(args, ranks, codec, dev, stream)
        if rank == 0:
            out.setdefault("legs", {})["compact_config4"] = c4
    if rank == 0:
        print(json.dumps(out), flush=True)
    ranks.close()


def _c4_fixture(rank, keys):
    if keys != 100_000:
        return None
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "compaction_configs.json")))
    return fx.get(f"config4_rank{rank}")


def compact4(args, ranks, codec, dev, stream):
    import shutil
    import tempfile
    td = tempfile.mkdtemp(prefix=f"sstc_bench_c4_r{ranks.rank}_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        make = lambda r: GpuCompaction(codec, dev, stream, td, W.config_inputs(4, r, keys=args.c4_keys),  # noqa: E731
                                       _c4_fixture(r, args.c4_keys))
        leg = config4_leg(ranks, make, args.c4_steps, lambda r: _c4_fixture(r, args.c4_keys))
        fx = _c4_fixture(ranks.rank, args.c4_keys)
        if ranks.world == 1 and fx is not None and not args.no_dropin:  # rank 0's shard through the unchanged caller
            sets = W.config_inputs(4, ranks.rank, keys=args.c4_keys)
            ranges = [record_key_range(r) for r in sets]
            del sets
            paths = [(os.path.join(td, f"in{i}.sst"), os.path.getsize(os.path.join(td, f"in{i}.sst")) + 1)
                     for i in range(len(ranges))]
            leg["dropin_rank0"] = dropin_leg(paths, ranges, fx, td, sum(fs - 1 for _, fs in paths))
    finally:
        shutil.rmtree(td, ignore_errors=True)
    bad = [p["rank"] for p in leg["per_rank"] if p["verified_vs_reference"] is False]
    if bad:
        raise SystemExit(f"config-4 leg: ranks {bad} produced outputs that differ from the reference's")
    leg["traffic_rank0"] = read_compact_traffic("config4")
    return leg


def plumbing(args, ranks):
    """The launcher / rank / timing / aggregation path of the bench without a
    GPU: each rank copies its shard's bytes on the host as its "step".  For
    the CPU test of `--gpus N` (tests/test_bench_launch.py); not a measurement."""
    nb = min(args.blocks, 256)
    a = np.full(nb * BLOCK_BYTES, ranks.rank, np.uint8)
    b = np.empty_like(a)
    ranks.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.copyto(b, a)
    ranks.barrier()
    wall = time.perf_counter() - t0
    per_rank = ranks.gather([wall, float(b[0])])
    wall_max = max(w for w, _ in per_rank)
    c4 = None
    if not args.no_compact4:  # the config-4 shard / rank / aggregation path with a host merge as the job
        keys = min(args.c4_keys, 64)
        c4 = config4_leg(ranks, lambda r: HostPlumbing(W.config_inputs(4, r, keys=keys)), 2, lambda r: None)
        c4["data"] = f"plumbing: 128 SSTs x {keys} records per rank, host merge of the key indices: not a measurement"
    if ranks.rank == 0:
        print(json.dumps({"metric": METRIC, "compact_config4": c4, "value": round(nb * BLOCK_BYTES * ranks.world * args.steps / wall_max
                                                          / 2 ** 30, 3),
                          "unit": "GiB/s", "n_gpus": ranks.world, "steps": args.steps, "warmup": args.warmup,
                          "scaling": "weak", "data": "plumbing check (host copy, gloo): not a measurement",
                          "per_rank": [{"rank": r, "shard_tag": int(t)} for r, (_, t) in enumerate(per_rank)]}),
              flush=True)
    ranks.close()


if __name__ == "__main__":
    main()
