#!/usr/bin/env python3
"""Benchmark of the MI355X DCT codec hot path (BASELINE.json `metric`).

A step = one DCT compress + decompress round trip of one batch of
--inflight x --batch (default 3 x 7 = 21) 4032x3008 IYUV frames (BASELINE.json
configs[1]: chef-with-trumpet-big, q=50; its raw input is missing from the
reference, so the frame is the decode of chef-with-trumpet-big-DCT-50.myyuv,
sha-pinned), with the frames and the compressed streams resident in HBM.
value = megapixels (luma W*H) of all ranks' frames / max-over-ranks wall time
of the K timed steps.  The frames are read from --input-frames (default 24)
distinct copies in HBM (436 MB, more than the 256 MiB Infinity Cache), so
every launch group reads its pixels from HBM, not from a cache-resident
buffer.

Batches and streams: a launch group of --batch frames (default 6) goes through
the batch entry points (one launch per kernel for all of them: a 4K frame is
too small to fill the MI355X, and every kernel's fixed launch and ramp time is
shared), and --inflight groups (default 3) are in flight on their own codec
contexts and HIP streams, so one group's latency-bound kernels (K2's overflow
pass, the chained scans) overlap another's work.  A step is still one frame:
value = frames x megapixels / wall time.

roofline: K1 fdct_quant (the block-transform kernel of the north star),
algorithmic bytes = 3 B per sample (1 B u8 in + 2 B int16 out) x W*H*3/2
samples per launch, divided by its average launch time from HIP events on the
launch stream over the timed region (where K1 shares the GPU with the other
frames in flight; the events ride on context 0's launches — one group in
--inflight, spread evenly over the region — since stamping every launch costs
~5 % of throughput); roofline_isolated: the same from the untimed one-frame-at-a-
time breakdown pass.  `traffic` = FETCH_SIZE*2 + WRITE_SIZE
per launch from a rocprofv3 --pmc run committed under profiles/ (null if none).

cpu_baseline: the reference library itself (oracle/_ref, built from the
reference sources with OpenMP, kind "reference") — or the C restatement
(oracle/, kind "port") when _ref is absent — timed on this box's host cores,
rank 0 at N=1 only, on a bounded sample of the same workload.

N>1: `python bench.py --gpus N` with no WORLD_SIZE in the environment starts
`torch.distributed.run --nproc-per-node N` as a child process before anything
touches a GPU and exits with its status; under a launcher WORLD_SIZE must
equal --gpus.  One rank per GPU: frames are sharded one per GPU
(weak scaling); inside the timed region rank 0 gathers every rank's
compressed streams over RCCL (batch.ChunkedGather: per chunk of frames the
sizes are all-gathered, then one packed exact-size point-to-point message per
rank, overlapped with the following chunks' compression): the batch
configuration's exchange step.
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "yuv-manipulations-2_amd")
sys.path[:0] = [ROOT, PKG]

GOLDEN_BIG = os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv")
BIG_DECODED_SHA = "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"
BIG_RECOMPRESSED_SHA = "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8 TB/s spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40,
                    help="timed steps; a step is one batch of --inflight x --batch frames")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--quality", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the cpu_baseline sample (0 disables it)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = OMP_NUM_THREADS or nproc")
    ap.add_argument("--events-ctx0", action="store_true",
                    help="event-stamp K1 on launch group 0 only (default: every group's K1 launches)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time the step without K1's HIP events (no roofline)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="frames in flight per GPU: steps rotate over this many codec contexts, "
                         "each on its own HIP stream, so one frame's latency-bound kernels overlap "
                         "another's (1 = strictly serial)")
    ap.add_argument("--batch", type=int, default=7,
                    help="frames per launch (the batch entry points): each kernel covers this "
                         "many frames")
    ap.add_argument("--stream-priority", default="",
                    help="comma-separated HIP stream priorities of the launch groups' streams "
                         "(cycled; default all normal)")
    ap.add_argument("--gather-chunk", type=int, default=32,
                    help="N>1: frames per chunk of the overlapped gather to rank 0")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the side measurements (decode-only rate, K7 BMP->IYUV roofline)")
    ap.add_argument("--breakdown-steps", type=int, default=5,
                    help="untimed launch groups after the timed region with every kernel stamped")
    ap.add_argument("--input-frames", type=int, default=24,
                    help="distinct HBM copies of the input frame the launch groups read in turn "
                         "(24 x 18.2 MB = 436 MB: larger than the 256 MiB Infinity Cache; rounded "
                         "down to a multiple of --batch: 21 copies, 382 MB, at the default 7)")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="only check the multi-rank launch: each rank joins a gloo group and "
                         "rank 0 prints the world size and an all_reduce (no GPU)")
    return ap.parse_args()


def maybe_launch(args):
    """--gpus N > 1 without a launcher: start N ranks with torch.distributed.run
    as a child process (nothing in this process has touched a GPU) and return
    its exit status.  Under a launcher, WORLD_SIZE must equal --gpus."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    log("bench.py: launching", " ".join(cmd))
    return subprocess.run(cmd).returncode


def launch_selftest():
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([dist.get_rank() + 1], dtype=torch.int64)
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "rank_sum": int(t.item())}), flush=True)
    dist.destroy_process_group()


def load_traffic(frame, batch):
    """Per-launch HBM bytes of K1 (calibrated FETCH_SIZE / WRITE_SIZE) from the
    newest profile of this bench workload (profiles/*_traffic.json written by
    tools/traffic.py from a tools/profile.sh run, which records the profiled
    frame and launch-group size), scaled to `batch` frames per launch."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    found = None
    for n in sorted(os.listdir(pdir)):
        if not n.endswith("_traffic.json"):
            continue
        try:
            with open(os.path.join(pdir, n)) as f:
                d = json.load(f)
            b = d.get("_bench") or {}
            v = d.get("fdct_quant", {}).get("hbm_bytes_per_launch")
            if b.get("frame") == frame and b.get("frames_per_launch") and v:
                found = v * batch // b["frames_per_launch"]
        except Exception:
            continue
    return found


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def usable_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count()


def cpu_baseline(raw, w, h, q, seconds, threads):
    """Reference OpenMP build (or the C restatement) on the host cores, plus
    the reference's serial build (its MYYUV_USE_OPENMP=OFF configuration,
    myyuv_lib/CMakeLists.txt:28-31) as the 1-thread figure."""
    nproc = usable_cpus()
    ncpu = threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or nproc
    os.environ["OMP_NUM_THREADS"] = str(ncpu)
    mp = w * h / 1e6
    host = {"cpu_model": cpu_model(), "cpus_visible": nproc}
    try:
        from oracle import ref as R
        if R.available("omp"):
            tc, td = R.bench(raw, w, h, (q, q, q), 1)
            iters = max(3, min(64, int(seconds / max(1e-3, (tc + td) / 1e3))))
            tc, td = R.bench(raw, w, h, (q, q, q), iters)
            one = None
            if R.available("serial"):
                sc, sd = R.bench(raw, w, h, (q, q, q), 5, variant="serial")
                one = {"value": round(mp / ((sc + sd) / 1e3), 2), "unit": "MP/s", "cores": 1,
                       "sample": f"5 round trips (median) of the same frame, reference serial build "
                                 f"(compress {sc:.1f} ms + decompress {sd:.1f} ms)"}
            return {"value": round(mp / ((tc + td) / 1e3), 2), "unit": "MP/s", "cores": ncpu,
                    "kind": "reference",
                    "sample": f"{iters} in-process compress+decompress round trips of the "
                              f"{w}x{h} q{q} frame (median; reference myyuv_lib -O3 OpenMP, "
                              f"compress {tc:.1f} ms + decompress {td:.1f} ms)",
                    "single_thread": one, **host}
    except Exception as e:  # fall back to the restatement
        log("cpu_baseline: reference build unavailable:", e)
    from oracle import oracle as O
    O.set_num_threads(ncpu)
    t0 = time.perf_counter()
    pay = O.compress(raw, w, h, (q, q, q))
    O.decompress(pay, w, h, (q, q, q))
    one = time.perf_counter() - t0
    iters = max(3, min(64, int(seconds / max(one, 1e-3))))
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        pay = O.compress(raw, w, h, (q, q, q))
        O.decompress(pay, w, h, (q, q, q))
        ts.append(time.perf_counter() - t0)
    ts.sort()
    t = ts[len(ts) // 2]
    return {"value": round(mp / t, 2), "unit": "MP/s", "cores": ncpu, "kind": "port",
            "sample": f"{iters} compress+decompress round trips of the {w}x{h} q{q} frame "
                      f"(median; C restatement -O2 OpenMP)", **host}


def main():
    args = parse()
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)
    if args.launch_selftest:
        launch_selftest()
        return
    import torch
    import myyuv_hip
    import myyuv_file

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    nf = max(1, args.inflight)
    codecs = [myyuv_hip.Codec(local) for _ in range(nf)]
    codec = codecs[0]

    # ---- workload: the decoded big golden frame (sha-pinned)
    g = myyuv_file.YUVFile.load(GOLDEN_BIG)
    w, h, q = g.width, g.height, args.quality
    raw = codec.decompress(g.data, w, h, tuple(g.params))
    if hashlib.sha256(g.decompressed(raw).dumps()).hexdigest() != BIG_DECODED_SHA:
        raise SystemExit("decoded chef-big frame does not match its pinned sha")
    mp = w * h / 1e6
    samples = w * h * 3 // 2
    cap = myyuv_hip.payload_bound(w, h)
    # a step = nf launch groups of B frames; launch group j runs on codec
    # context j % nf and its own stream (contexts own their scratch buffers,
    # so groups in flight never share one)
    B = max(1, args.batch)
    per_step = nf * B
    frames = args.steps * per_step
    # explicit streams: the null stream's handle is 0, which the C ABI reads as
    # "the context's own stream" (the N>1 gather's events must see the launches)
    # --stream-priority: per launch group, a HIP stream priority (0 normal,
    # negative higher), cycled over the groups in flight
    prios = [int(v) for v in args.stream_priority.split(",")] if args.stream_priority else [0]
    streams = [torch.cuda.Stream(dev, priority=prios[k % len(prios)]) for k in range(nf)]
    sps = [st.cuda_stream for st in streams]
    cap = (cap + 3) & ~3  # payload slots of a batch are dword aligned
    # distinct input copies (HBM-resident, more than the Infinity Cache holds);
    # launch group j reads copies (j*B .. j*B+B-1) mod nin
    nin = max(B, (max(args.input_frames, B) // B) * B)
    d_in = torch.empty((nin, samples), dtype=torch.uint8, device=dev)
    d_in[:] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    for st in streams:
        st.wait_stream(torch.cuda.current_stream(dev))
    ingroups = nin // B
    d_out = torch.empty((nf, B * samples), dtype=torch.uint8, device=dev)
    # one payload slot per timed frame: the batch of compressed streams this
    # rank contributes (gathered to rank 0 at N>1)
    nslot = max(frames, per_step * max(1, args.warmup))
    d_pay = torch.empty((nslot, cap), dtype=torch.uint8, device=dev)
    d_size = torch.zeros(nslot, dtype=torch.int32, device=dev)
    for c in codecs:
        c.reserve_batch(w, h, B)
    slot_groups = nslot // B

    def group(j, nb=B):
        k = j % nf
        f0 = (j % slot_groups) * B
        src = d_in[(j % ingroups) * B].data_ptr()
        codecs[k].compress_batch_device(src, nb, w, h, (q, q, q), d_pay[f0].data_ptr(), cap,
                                        d_size[f0:f0 + nb].data_ptr(), sps[k])
        codecs[k].decompress_batch_device(d_pay[f0].data_ptr(), d_size[f0:f0 + nb].data_ptr(), cap, nb,
                                          w, h, (q, q, q), d_out[k].data_ptr(), sps[k])

    def check_status():
        for k, c in enumerate(codecs):
            rc, bad = c.sync_status(sps[k])
            if rc:
                raise SystemExit(f"codec error {rc} ({myyuv_hip.strerror(rc)}) at block {bad}")

    for j in range(max(1, args.warmup) * nf):
        group(j)
    check_status()
    n0 = int(d_size[0].item())
    pay0 = bytes(d_pay[0, :n0].cpu().numpy())
    if q == 50 and hashlib.sha256(pay0).hexdigest() != BIG_RECOMPRESSED_SHA:
        raise SystemExit("compressed stream differs from the pinned reference bytes")
    host_rt = codec.decompress(pay0, w, h, (q, q, q))
    for f in range(per_step):
        nk = int(d_size[f].item())
        if bytes(d_pay[f, :nk].cpu().numpy()) != pay0:
            raise SystemExit(f"frame slot {f}: compressed stream differs from slot 0's")
    for k in range(nf):
        for b in range(B):
            if bytes(d_out[k, b * samples:(b + 1) * samples].cpu().numpy()) != host_rt:
                raise SystemExit(f"context {k} frame {b}: device round trip differs from the host-API decode")

    # ---- timed region: only K1 (the roofline kernel) is event-stamped, on
    # every launch group (so the average is over the same launches a
    # rocprofv3 kernel trace of this run averages), or on launch group 0 only
    # (--events-ctx0)
    stamped = codecs[:1] if args.events_ctx0 else codecs
    if not args.no_kernel_events:
        for c in stamped:
            c.profile(True, kernels=["fdct_quant"])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    # N>1: the batch's exchange step, every rank's compressed streams to rank 0
    # (batch.ChunkedGather): chunks of --gather-chunk frames; a chunk's sizes
    # are all-gathered when its launch groups are done and its streams sent
    # while the following chunks compute
    gat = None
    if world > 1:
        import batch
        gat = batch.ChunkedGather(dist, world, rank, dev)
    cg = max(1, args.gather_chunk // B)  # launch groups per chunk
    ngr = args.steps * nf
    evs, c0 = [], 0
    for j in range(ngr):
        group(j)
        if gat is not None:
            ev = torch.cuda.Event()
            ev.record(streams[j % nf])
            evs.append(ev)
            if len(evs) == cg or j == ngr - 1:
                i1 = (j + 1) * B
                gat.add(list(range(c0, i1)), [d_pay[i] for i in range(c0, i1)], d_size[c0:i1], evs)
                evs, c0 = [], i1
    for st in streams:
        torch.cuda.current_stream(dev).wait_stream(st)
    gathered = None
    if gat is not None:
        got = gat.finish(frames)
        gathered = sum(t is not None for t in got) if got is not None else 0
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    check_status()
    stats = {}
    if not args.no_kernel_events:
        for c in stamped:
            for kname, (kms, kn) in c.kernel_stats().items():
                a, n = stats.get(kname, (0.0, 0))
                stats[kname] = (a + kms, n + kn)
            c.profile(False)
    # per-kernel breakdown (all kernels stamped, one launch group at a time on
    # one stream), outside the timed region
    breakdown = {}
    if args.breakdown_steps > 0:
        codec.profile(True)
        for i in range(args.breakdown_steps):
            group(i * nf)
        codec.sync_status(sps[0])
        breakdown = codec.kernel_stats()
        codec.profile(False)
    # side measurements, outside the timed region
    side = None
    if rank == 0 and not args.no_side:
        side = {}
        # decode-only batched rate: the same launch groups, decompress only,
        # from the streams the timed region left in HBM

        def dgroup(j):
            k = j % nf
            f0 = (j % (frames // B)) * B
            codecs[k].decompress_batch_device(d_pay[f0].data_ptr(), d_size[f0:f0 + B].data_ptr(), cap, B,
                                              w, h, (q, q, q), d_out[k].data_ptr(), sps[k])
        nd = ngr
        for j in range(nf):
            dgroup(j)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for j in range(nd):
            dgroup(j)
        for st in streams[1:]:
            streams[0].wait_stream(st)
        torch.cuda.synchronize(dev)
        td = time.perf_counter() - t0
        check_status()
        side["decode_only"] = {"value": round(nd * B * mp / td, 2), "unit": "MP/s", "frames": nd * B}
        # K7 BMP -> IYUV on a 4032x3008 BGRA bottom-up frame: 4 B in + 1.5 B out
        # per pixel, streaming, so its bound is HBM
        bgra = torch.randint(0, 256, (w * h * 4,), dtype=torch.uint8, device=dev)
        d_iy = torch.empty(w * h * 3 // 2, dtype=torch.uint8, device=dev)
        sp0 = sps[0]
        for _ in range(3):
            codec.bmp_to_iyuv_device(bgra.data_ptr(), w, h, 32, d_iy.data_ptr(), sp0)
        codec.sync_status(sp0)
        codec.profile(True, kernels=["bmp_to_iyuv"])
        for _ in range(50):
            codec.bmp_to_iyuv_device(bgra.data_ptr(), w, h, 32, d_iy.data_ptr(), sp0)
        codec.sync_status(sp0)
        kms, kn = codec.kernel_stats()["bmp_to_iyuv"]
        codec.profile(False)
        if kn:
            alg = w * h * 4 + w * h * 3 // 2
            a7 = alg / (kms / kn * 1e-3) / 1e9
            side["bmp_to_iyuv"] = {"bound": "hbm", "achieved": round(a7, 1), "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(a7 / HBM_PEAK_GBS, 4),
                                   "algorithmic_bytes_per_launch": alg,
                                   "avg_launch_us": round(kms / kn * 1e3, 2), "frame": f"{w}x{h} BGRA"}
        del bgra, d_iy
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
        if rank == 0:
            assert gathered == world * frames, gathered

    if rank == 0:
        ms_step = t / args.steps * 1e3
        value = world * frames * mp / t
        k1_ms, k1_n = stats.get("fdct_quant", (0.0, 0))
        roof = None
        if k1_n:
            avg_s = k1_ms / k1_n / 1e3
            alg = round(3 * samples * B)  # a launch covers a batch of B frames
            achieved = alg / avg_s / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": load_traffic(f"{w}x{h}", B), "kernel": "fdct_quant",
                    "algorithmic_bytes_per_launch": alg, "avg_launch_us": round(avg_s * 1e6, 2)}
        kernel_us = {k: round(kms / kn * 1e3, 2) for k, (kms, kn) in breakdown.items() if kn}
        # the same K1 figure with one launch group at a time (the untimed
        # breakdown pass): the kernel alone on the GPU, no co-running group
        roof_iso = None
        if roof and kernel_us.get("fdct_quant"):
            a_iso = 3 * samples * B / (kernel_us["fdct_quant"] * 1e-6) / 1e9
            roof_iso = {"achieved": round(a_iso, 1), "frac": round(a_iso / HBM_PEAK_GBS, 4),
                        "avg_launch_us": kernel_us["fdct_quant"]}
        # K6 (dequant + inverse DCT, 2 B in + 1 B out per sample) the same way
        roof_k6 = None
        if kernel_us.get("dequant_idct"):
            a6 = 3 * samples * B / (kernel_us["dequant_idct"] * 1e-6) / 1e9
            roof_k6 = {"kernel": "dequant_idct", "achieved": round(a6, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(a6 / HBM_PEAK_GBS, 4),
                       "algorithmic_bytes_per_launch": 3 * samples * B,
                       "avg_launch_us": kernel_us["dequant_idct"]}
        # the fused decoder (default; K5 + K6 in one kernel, the "huff_decode"
        # id): stream bytes in + 1 B per sample out
        roof_dec = None
        if not kernel_us.get("dequant_idct") and kernel_us.get("huff_decode"):
            alg_d = (n0 + samples) * B
            ad = alg_d / (kernel_us["huff_decode"] * 1e-6) / 1e9
            roof_dec = {"kernel": "decode_idct (fused K5+K6)", "achieved": round(ad, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ad / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg_d,
                        "avg_launch_us": kernel_us["huff_decode"]}
        for k, us in kernel_us.items():
            log(f"kernel {k:16s} {us:9.2f} us/launch")
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            cpu = cpu_baseline(raw, w, h, q, args.cpu_seconds, args.cpu_threads)
        line = {
            "metric": "megapixels/sec DCT compress+decompress, 4K IYUV; achieved HBM GB/s vs peak",
            "value": round(value, 2), "unit": "MP/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/int16 (fp32 transform)",
            "data": "chef-with-trumpet-big-DCT-50.myyuv decoded (4032x3008 IYUV, sha-pinned); "
                    f"stand-in for the missing raw 4K; {nin} distinct HBM copies",
            "config": {"workload": f"chef-with-trumpet-big 4032x3008 IYUV DCT q={q} "
                                   f"compress+decompress, HBM-resident, {per_step} frames/step/GPU",
                       "frame": f"{w}x{h}", "quality": q, "parallelism": f"frames sharded, dp{world}",
                       "frames_per_step": per_step, "launch_groups_in_flight": nf,
                       "frames_per_launch": B, "input_copies": nin, "payload_bytes": n0},
            "roofline": roof, "roofline_isolated": roof_iso, "roofline_idct_isolated": roof_k6,
            "roofline_decode_isolated": roof_dec,
            "cpu_baseline": cpu,
            "kernel_us": kernel_us or None,
            "side": side,
        }
        print(json.dumps(line), flush=True)
    for c in codecs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
