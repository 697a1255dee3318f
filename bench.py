#!/usr/bin/env python3
"""Benchmark of the MI355X DCT codec hot path (BASELINE.json `metric`).

Workloads (--workload; `auto`, the default, is chef-big at every rank count,
so the driver's 1/2/4/8-GPU runs form one weak-scaling curve of one workload):
  chef-big  BASELINE.json configs[1], the metric's own configuration: a step
            is one DCT compress + decompress round trip of --inflight x
            --batch (default 4 x 32 = 128) 4032x3008 IYUV frames per rank
            (chef-with-trumpet-big, q=50; its raw input is missing from the
            reference, so the frame is the sha-pinned decode of
            chef-with-trumpet-big-DCT-50.myyuv), read from --input-frames
            (default: one per frame of a step, at least 32, rounded down to a
            multiple of --batch) distinct HBM copies: more bytes than the 256
            MiB Infinity Cache, so the pixel reads come from HBM.  Weak scaling: every rank runs that batch,
            and at N > 1 every rank's compressed streams are gathered to rank 0
            inside the timed region (rank 0 checks the first, middle and last).
  batch4k   BASELINE.json configs[3]/[4]: a step is the batch of --frames
            (default 512) synthetic 3840x2160 IYUV frames, q=50 (frame f: the
            tiled chef-big frame with origin (8f mod 4032, 8f mod 3008),
            SURVEY.md §8d), dealt round-robin over the ranks (frame f on rank
            f mod N), compressed and decompressed where they live; at N > 1
            every rank's compressed streams are gathered to rank 0 inside the
            timed region.  The batch is fixed, so at N ranks each rank runs
            --frames / N frames: strong scaling.  Checked against
            tests/golden/batch4k_512.json (the oracle's payload and decode
            sha256 per frame): every stream and every decode of the untimed
            first pass, and at N > 1 every gathered stream of the first and
            the last timed step (the timed region's decodes are not compared).
            At the default chef-big workload the same batch runs after the
            timed region on all ranks as `side.batch4k` (at every N, so that
            line is a strong-scaling curve of its own).
value = megapixels (luma W*H) of all ranks' frames / max-over-ranks wall time
of the K timed steps; frames and streams stay in HBM.  At N > 1 the line also
carries `ranks`: per rank its wall time, its compute time (HIP events from the
start of the timed region to the end of its last launch group), the exposed
gather tail (wall - compute) and the stream bytes it sent (rank 0: received).
Every rank's status (its codec's device errors, a payload past its slot) is
all-gathered after the untimed pass and after the timed region; one failing
rank makes every rank exit non-zero.

Execution: launch groups of --batch frames go through the batch entry points
(one launch per kernel covers the group), and --inflight groups are in flight
on their own codec contexts and explicit HIP streams, so one group's
latency-bound kernels (the overflow pass, the chained scans) overlap
another's work.  Launch group i of a batch4k step always runs on context
i mod --inflight (its payload slots are reused from step to step in stream
order at N = 1).

roofline: K1 fdct_quant, the block-transform kernel of the north star.
Algorithmic bytes = 3 B per sample (1 B u8 in + 2 B int16 out)
x the samples of the launches; time = those launches' HIP-event durations,
K1's own; k_fdct_fix (K1's exact path for the blocks whose fast result it
cannot prove; it runs right after K1 in the stream) is stamped as well and
reported beside it, with the fraction of K1 + fix summed (`fix_kernel`)
(dispatch-stamped on their streams, every launch group's K1 by default,
--events-ctx0: group 0's only) over the timed region, where K1 shares the GPU
with the other groups in flight.  `traffic` = calibrated FETCH_SIZE/WRITE_SIZE
bytes per launch from the newest rocprofv3 --pmc profile of this workload
under profiles/ (null if none); `traffic_gbs` = traffic / avg launch time.
K1 is VALU-issue bound: `valu_ceiling_frac` is the fraction of
the HBM peak its fast path's instructions alone allow (the gfx950 code object's
loop body weighted by the measured issue cost of each instruction form,
K1_ISSUE_NS_PER_UNIT, on 1,024 SIMDs), so `frac` reads against it.  roofline_isolated: the
same K1 figure from the untimed one-group-at-a-time breakdown pass.

cpu_baseline (rank 0, N = 1): the reference library itself (oracle/_ref,
built from the reference sources with OpenMP, kind "reference") — or the C
restatement (oracle/, kind "port") when _ref is absent — on a bounded sample
of the same workload, with all usable host cores (the process's CPU affinity
bounded by the cgroup CPU quota, both reported), plus the box's per-GPU CPU
share (OMP_NUM_THREADS as the box sets it) and the reference's serial build.

side (rank 0, outside the timed region): decode_only (the same launch groups
decompress only), bmp_to_iyuv (K7's roofline), host_api (the host-buffer
C ABI a reference-side plugin calls, myyuv_gpu_dct_compress +
myyuv_gpu_dct_decompress on the chef-big frame: time = t_compress +
t_decompress, PCIe included), and at N = 1 with the chef-big
workload, batch4k: the configs[3] batch on this one GPU (the N = 1 point of
that workload's scaling curve).

N>1: `python bench.py --gpus N` with no WORLD_SIZE in the environment starts
`torch.distributed.run --nproc-per-node N` as a child process before anything
touches a GPU and exits with its status; under a launcher WORLD_SIZE must
equal --gpus.  One rank per GPU; rank 0 gathers every rank's compressed
streams over RCCL (batch.ChunkedGather: per chunk of --gather-chunk frames the
sizes are all-gathered, then one packed exact-size point-to-point message per
rank, overlapped with the following chunks' work).

--cpu-codec (tests only): the CPU restatement (oracle/) stands in for the HIP
codec, on host tensors over gloo, so the whole N > 1 loop — sharding, launch
groups, the chunked gather, the checks — runs on a machine without a GPU.  Its
`value` is not a measurement of the product.
"""
import argparse
import hashlib
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "yuv-manipulations-2_amd")
sys.path[:0] = [ROOT, PKG]

GOLDEN_BIG = os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv")
MANIFEST_4K = os.path.join(ROOT, "tests", "golden", "batch4k_512.json")
BIG_DECODED_SHA = "5e7769191188285cc127c6b4da900b3420f064191f707383c82128c14e497e5c"
BIG_RECOMPRESSED_SHA = "fe9b7317653c2b44a9f24436f0e349b083b4e368cf9653e8777e9f7a79cebfcc"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8 TB/s spec)
SLOT_4K = 4 << 20  # batch4k payload slot: the largest of the 512 streams is 2,471,404 B (capacity is checked on device)
# K1's VALU issue time: the fast path's loop body in the
# gfx950 code object of this build, weighted by the issue cost of each
# instruction form measured on MI355X at 8 waves per SIMD (tools/ubench/
# vforms.hip, iforms.hip; profiles/r6g_iforms_and_k5_forms.txt): 1.0 ns per
# wave-instruction per SIMD for the VOP2/VOP1 forms and f32 mul/add/fma,
# 1.8 ns for VOP3-only integer forms, compares, conversions, SDWA, DPP and
# packed forms.  Round 6: 246 fast + 131 slow instructions per lane-unit
# (round 5's flat stores: 254 + 144)
K1_ISSUE_NS_PER_UNIT = 246 * 1.0 + 131 * 1.8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40,
                    help="timed steps; chef-big: --inflight x --batch frames per rank, batch4k: the --frames batch")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--workload", choices=("auto", "chef-big", "batch4k"), default="auto",
                    help="auto: chef-big (configs[1]) at every rank count (side.batch4k runs configs[3])")
    ap.add_argument("--frames", type=int, default=512,
                    help="batch4k: frames per step over all ranks (a multiple of the rank count)")
    ap.add_argument("--quality", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget of the cpu_baseline sample (0 disables it)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="cpu_baseline threads (0 = all usable cores: affinity bounded by the cgroup quota)")
    ap.add_argument("--events-ctx0", action="store_true",
                    help="event-stamp K1 on launch group 0 only (default: every group's K1 launches)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time the step without K1's HIP events (no roofline)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="launch groups in flight per GPU, each on its own codec context and HIP stream "
                         "(1 = strictly serial; 0 = 4)")
    ap.add_argument("--batch", type=int, default=0,
                    help="frames per launch (the batch entry points; 0 = 32 for chef-big, 24 for batch4k)")
    ap.add_argument("--stream-priority", default="",
                    help="comma-separated HIP stream priorities of the launch groups' streams "
                         "(cycled; default all normal)")
    ap.add_argument("--gather-chunk", type=int, default=32,
                    help="N>1: frames per chunk of the overlapped gather to rank 0")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the side measurements (decode-only, K7 roofline, host API, batch4k at N=1)")
    ap.add_argument("--host-api-iters", type=int, default=20,
                    help="round trips of the host-buffer API side measurement (0 disables it)")
    ap.add_argument("--host-batch-frames", type=int, default=32,
                    help="frames of the pipelined host-buffer batch side measurement (0 disables it)")
    ap.add_argument("--breakdown-steps", type=int, default=5,
                    help="untimed launch groups after the timed region with every kernel stamped")
    ap.add_argument("--input-frames", type=int, default=0,
                    help="chef-big: distinct HBM copies of the input frame the launch groups read in turn "
                         "(0: one per frame of a step, at least 32; rounded down to a multiple of --batch: "
                         "128 copies, 2.33 GB at the default 4 x 32, larger than the 256 MiB Infinity Cache)")
    ap.add_argument("--cpu-codec", action="store_true",
                    help="tests only: the CPU restatement as the codec, host tensors, gloo (no GPU)")
    ap.add_argument("--cpu-codec-fail", default="",
                    help="tests only, with --cpu-codec: RANK:WHERE (warmup|timed) makes that rank's codec "
                         "report an error there (timed: its first stream also gets a size past its slot)")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="only check the multi-rank launch: each rank joins a gloo group and "
                         "rank 0 prints the world size and an all_reduce (no GPU)")
    return ap.parse_args(argv)


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


def cgroup_cpu_quota():
    """CPUs the cgroup CPU quota allows (cgroup v2 cpu.max, v1
    cpu.cfs_quota_us / cfs_period_us), as (cpus or None for no limit, source)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return (None if q == "max" else int(q) / int(p)), f"cgroup v2 cpu.max '{q} {p}'"
    except (OSError, ValueError):
        pass
    for d in ("/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
        try:
            with open(os.path.join(d, "cpu.cfs_quota_us")) as f:
                q = int(f.read())
            with open(os.path.join(d, "cpu.cfs_period_us")) as f:
                p = int(f.read())
            return (None if q <= 0 else q / p), f"cgroup v1 cfs_quota_us {q} / cfs_period_us {p}"
        except (OSError, ValueError):
            continue
    return None, "no cgroup CPU controller found"


def usable_cpus():
    """(usable cores, affinity count, quota cpus, quota source): the process's
    CPU affinity bounded by the cgroup quota."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    quota, src = cgroup_cpu_quota()
    use = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    return use, aff, quota, src


def cpu_baseline(raw, w, h, q, seconds, threads):
    """Reference OpenMP build (or the C restatement) on the host cores: all
    usable cores, the box's per-GPU share (OMP_NUM_THREADS as set on the box)
    and the reference's serial build (its MYYUV_USE_OPENMP=OFF configuration,
    myyuv_lib/CMakeLists.txt:28-31)."""
    use, aff, quota, qsrc = usable_cpus()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    ncpu = threads or use
    mp = w * h / 1e6
    host = {"cpu_model": cpu_model(), "cpus_visible": os.cpu_count(), "cpus_affinity": aff,
            "cgroup_quota": quota, "cgroup_quota_source": qsrc, "usable_cores": use}

    old = os.environ.get("OMP_NUM_THREADS")
    try:
        from oracle import ref as R
        if R.available("omp"):
            # (each run in its own process: libgomp reads OMP_NUM_THREADS once per process)
            tc, td, iters = _ref_in_child(raw, w, h, q, ncpu, seconds, "omp")
            out = {"value": round(mp / ((tc + td) / 1e3), 2), "unit": "MP/s", "cores": ncpu,
                   "kind": "reference",
                   "sample": f"{iters} in-process compress+decompress round trips of the {w}x{h} q{q} frame "
                             f"(median; reference myyuv_lib -O3 OpenMP, {ncpu} threads: "
                             f"compress {tc:.1f} ms + decompress {td:.1f} ms)", **host}
            if share and share != ncpu:
                sc, sd, si = _ref_in_child(raw, w, h, q, share, seconds / 2, "omp")
                out["box_share"] = {"value": round(mp / ((sc + sd) / 1e3), 2), "unit": "MP/s", "cores": share,
                                    "sample": f"{si} round trips, {share} threads (the box's per-GPU CPU share, "
                                              f"OMP_NUM_THREADS)"}
            if R.available("serial"):
                sc, sd, _ = _ref_in_child(raw, w, h, q, 1, 0, "serial", iters=5)
                out["single_thread"] = {"value": round(mp / ((sc + sd) / 1e3), 2), "unit": "MP/s", "cores": 1,
                                        "sample": f"5 round trips (median) of the same frame, reference serial "
                                                  f"build (compress {sc:.1f} ms + decompress {sd:.1f} ms)"}
            return out
    except Exception as e:  # fall back to the restatement
        log("cpu_baseline: reference build unavailable:", e)
    finally:
        if old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = old
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


def _ref_in_child(raw, w, h, q, threads, seconds, variant, iters=0):
    """Times the reference library in a child process with OMP_NUM_THREADS =
    threads (libgomp fixes its team size when it loads); returns medians
    (compress ms, decompress ms, iterations)."""
    import subprocess
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".iyuv", delete=False) as f:
        f.write(raw)
        path = f.name
    try:
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        code = ("import sys; sys.path.insert(0, %r)\n"
                "from oracle import ref as R\n"
                "raw = open(%r, 'rb').read(); w, h, q, budget, n = %d, %d, %d, %f, %d\n"
                "if not n:\n"
                "    tc, td = R.bench(raw, w, h, (q, q, q), 1, variant=%r)\n"
                "    n = max(3, min(64, int(budget / max(1e-3, (tc + td) / 1e3))))\n"
                "tc, td = R.bench(raw, w, h, (q, q, q), n, variant=%r)\n"
                "print(tc, td, n)\n") % (ROOT, path, w, h, q, seconds, iters, variant, variant)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
        if r.returncode:
            raise RuntimeError(r.stderr[-500:])
        tc, td, n = r.stdout.split()[-3:]
        return float(tc), float(td), int(n)
    finally:
        os.unlink(path)


# ---------------------------------------------------------------------------
# codecs: the HIP codec (the product) and, for the CPU tests of the loop, the
# C restatement on host tensors
# ---------------------------------------------------------------------------

class GpuCodec:
    """The HIP codec through the C ABI (myyuv_hip): one codec context and one
    explicit HIP stream per launch group in flight (the null stream's handle
    is 0, which the C ABI reads as "the context's own stream", and the gather's
    events must see the launches)."""

    def __init__(self, dev, nf, prios):
        import torch
        import myyuv_hip
        self.torch, self.dev = torch, dev
        self.codecs = [myyuv_hip.Codec(dev.index) for _ in range(nf)]
        self.streams = [torch.cuda.Stream(dev, priority=prios[k % len(prios)]) for k in range(nf)]
        self.sps = [st.cuda_stream for st in self.streams]

    def empty(self, shape, dtype=None):
        return self.torch.empty(shape, dtype=dtype or self.torch.uint8, device=self.dev)

    def reserve(self, w, h, B):
        for c in self.codecs:
            c.reserve_batch(w, h, B)

    def settle(self):
        for st in self.streams:
            st.wait_stream(self.torch.cuda.current_stream(self.dev))

    def compress(self, k, src, nb, w, h, q, pay, cap, size):
        self.codecs[k].compress_batch_device(src.data_ptr(), nb, w, h, q, pay.data_ptr(), cap, size.data_ptr(),
                                             self.sps[k])

    def decompress(self, k, pay, size, cap, nb, w, h, q, out):
        self.codecs[k].decompress_batch_device(pay.data_ptr(), size.data_ptr(), cap, nb, w, h, q, out.data_ptr(),
                                               self.sps[k])

    def event(self, k):
        ev = self.torch.cuda.Event()
        ev.record(self.streams[k])
        return ev

    def check(self):
        import myyuv_hip
        for k, c in enumerate(self.codecs):
            rc, bad = c.sync_status(self.sps[k])
            if rc:
                raise SystemExit(f"codec error {rc} ({myyuv_hip.strerror(rc)}) at block {bad}")

    def marker(self):
        """An event on the current stream (after join(): the end of every
        launch group enqueued so far)."""
        ev = self.torch.cuda.Event(enable_timing=True)
        ev.record(self.torch.cuda.current_stream(self.dev))
        return ev

    def join(self):
        for st in self.streams:
            self.torch.cuda.current_stream(self.dev).wait_stream(st)

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def close(self):
        for c in self.codecs:
            c.close()


class CpuCodec:
    """Tests only: the C restatement (oracle/) behind GpuCodec's interface, on
    host tensors, synchronous (no events)."""

    def __init__(self, nf, fail="", rank=0):
        import torch
        from oracle import oracle as O
        self.torch, self.O = torch, O
        self.streams = [None] * nf
        r, _, where = fail.partition(":")
        self.fail = where if fail and int(r) == rank else ""
        self.phase = "warmup"

    def empty(self, shape, dtype=None):
        return self.torch.empty(shape, dtype=dtype or self.torch.uint8)

    def reserve(self, w, h, B):
        pass

    def settle(self):
        pass

    def compress(self, k, src, nb, w, h, q, pay, cap, size):
        fb = w * h * 3 // 2
        for b in range(nb):
            p = self.O.compress(src[b].numpy(), w, h, q)
            if len(p) > cap:
                raise SystemExit("codec error 5 (Output buffer too small for the compressed stream)")
            pay[b, :len(p)] = self.torch.frombuffer(bytearray(p), dtype=self.torch.uint8)
            size[b] = len(p)
        if self.fail == "timed" and self.phase == "timed":
            size[0] = cap + 4096  # a size past its slot: the gather must not hang on it

    def decompress(self, k, pay, size, cap, nb, w, h, q, out):
        fb = w * h * 3 // 2
        flat = out.reshape(-1)
        for b in range(nb):
            d = self.O.decompress(pay[b, :int(size[b])].numpy().tobytes(), w, h, q)
            flat[b * fb:(b + 1) * fb] = self.torch.frombuffer(bytearray(d), dtype=self.torch.uint8)

    def event(self, k):
        return None

    def check(self):
        if self.fail and self.fail == self.phase:
            raise SystemExit("codec error 5 (Output buffer too small for the compressed stream) "
                             "[--cpu-codec-fail]")

    def marker(self):
        return None

    def join(self):
        pass

    def sync(self):
        pass

    def close(self):
        pass


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------

class Run:
    """One workload on this rank: its input frames, payload slots and launch
    groups.  group (s, i) = launch group i of step s: codec context k, its
    first input frame, its frame count, its first payload slot; at N > 1 the
    slot index is also the frame's local index in the gather (local frame j of
    rank r = global frame r + N * j, batch.ChunkedGather)."""

    def __init__(self, name, codec, raw, big, args, world, rank):
        import torch
        self.name, self.codec, self.world, self.rank = name, codec, world, rank
        self.q = args.quality
        self.q3 = (self.q, self.q, self.q)
        self.nf = len(codec.streams)
        self.verified = {}
        if name == "chef-big":
            self.w, self.h = big.width, big.height
            self.B = args.batch or 32
            self.per_step = self.nf * self.B
            self.n_local = self.per_step
            self.n_total = world * self.per_step
            self.cap = SLOT_4K if isinstance(codec, CpuCodec) else None
            want = args.input_frames or max(32, self.per_step)
            nin = max(self.B, (max(want, self.B) // self.B) * self.B)
            self.nin = nin
            self.samples = self.w * self.h * 3 // 2
            self.d_in = codec.empty((nin, self.samples))
            self.d_in[:] = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.d_in.device)
            self.ngroups = self.nf
            self.scaling = "weak"
        else:
            man = load_manifest()
            self.w, self.h = man["width"], man["height"]
            if self.q != man["quality"]:
                raise SystemExit(f"batch4k is configs[3]: q={man['quality']}")
            self.n_total = args.frames
            if self.n_total < world or self.n_total % world or self.n_total > man["frames_total"]:
                raise SystemExit(f"--frames {self.n_total}: a multiple of the {world} ranks, at most "
                                 f"{man['frames_total']}")
            self.B = args.batch or 24
            self.n_local = self.n_total // world
            self.per_step = self.n_local
            self.cap = SLOT_4K
            self.samples = self.w * self.h * 3 // 2
            self.ngroups = (self.n_local + self.B - 1) // self.B
            self.manifest = man["frames"]
            self.gframes = list(range(rank, self.n_total, world))
            import synth
            src = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
            if not isinstance(codec, CpuCodec):
                src = src.to(codec.dev)
            self.d_in = codec.empty((self.n_local, self.samples))
            for j, f in enumerate(self.gframes):
                ox, oy = synth.batch_origin(f, big.width, big.height)
                self.d_in[j] = synth.tiled_frame_torch(src, big.width, big.height, self.w, self.h, ox, oy)
            # every input frame against the manifest's input sha (the generator)
            bad = [f for f, d in zip(self.gframes, hashes(self.d_in, self.n_local))
                   if d != self.manifest[f]["input_sha"]]
            if bad:
                raise SystemExit(f"batch4k: generated frames {bad[:4]} differ from the manifest")
            self.scaling = "strong"
        if self.cap is None:
            import myyuv_hip
            self.cap = (myyuv_hip.payload_bound(self.w, self.h) + 3) & ~3  # batch slots are dword aligned
        self.mp = self.w * self.h / 1e6
        codec.reserve(self.w, self.h, self.B)
        self.d_out = codec.empty((self.nf, self.B * self.samples))

    def alloc_slots(self, steps, warmup):
        if self.name == "chef-big":
            nslot = max(steps * self.per_step, self.per_step * max(1, warmup))
        else:
            # (N > 1: one slot set per step, the gather reads them after the
            # step's launches; N = 1: one set, reused in stream order)
            nslot = self.n_local * (max(steps, warmup, 1) if self.world > 1 else 1)
        self.nslot = nslot
        self.d_pay = self.codec.empty((nslot, self.cap))
        self.d_size = self.codec.empty(nslot, dtype=self.codec.torch.int32)
        self.d_size.zero_()
        self.codec.settle()

    def group_desc(self, j):
        """Launch group j (counted over steps): (k, input row, frames, slot)."""
        s, i = divmod(j, self.ngroups)
        if self.name == "chef-big":
            k = j % self.nf
            src = (j % (self.nin // self.B)) * self.B
            slot = (j % (self.nslot // self.B)) * self.B
            return k, src, self.B, slot
        nb = min(self.B, self.n_local - i * self.B)
        slot = (s * self.n_local if self.world > 1 else 0) + i * self.B
        return i % self.nf, i * self.B, nb, slot

    def run_group(self, j, decompress=True, ctx=None):
        k, src, nb, slot = self.group_desc(j)
        if ctx is not None:
            k = ctx
        c = self.codec
        c.compress(k, self.d_in[src:src + nb], nb, self.w, self.h, self.q3, self.d_pay[slot:slot + nb], self.cap,
                   self.d_size[slot:slot + nb])
        if decompress:
            c.decompress(k, self.d_pay[slot:slot + nb], self.d_size[slot:slot + nb], self.cap, nb, self.w, self.h,
                         self.q3, self.d_out[k])
        return k, nb, slot

    def decode_group(self, j):
        k, _, nb, slot = self.group_desc(j)
        self.codec.decompress(k, self.d_pay[slot:slot + nb], self.d_size[slot:slot + nb], self.cap, nb, self.w,
                              self.h, self.q3, self.d_out[k])

    def warmup(self, passes):
        """passes x one step, untimed; the first pass is checked: chef-big,
        every stream against the pinned reference bytes and every round trip
        against the host-API decode (GPU); batch4k, group by group, every
        stream and its decode against the manifest."""
        c = self.codec
        n = max(1, passes) * self.ngroups
        if self.name == "batch4k":
            for j in range(self.ngroups):
                k, nb, slot = self.run_group(j)
                c.sync()
                sizes = self.d_size[slot:slot + nb].cpu().tolist()
                pays = [bytes(self.d_pay[slot + b, :sizes[b]].cpu().numpy()) for b in range(nb)]
                decs = hashes(self.d_out[k], nb, self.samples)
                for b in range(nb):
                    f = self.gframes[j * self.B + b]
                    m = self.manifest[f]
                    if len(pays[b]) != m["payload_size"] or sha(pays[b]) != m["payload_sha"]:
                        raise SystemExit(f"batch4k frame {f}: compressed stream differs from the manifest")
                    if decs[b] != m["decoded_sha"]:
                        raise SystemExit(f"batch4k frame {f}: decode differs from the manifest")
            c.check()
            self.verified["first_pass"] = (f"{self.n_local} frames on rank {self.rank}: payload size + sha256 and "
                                           f"decoded sha256 == tests/golden/batch4k_512.json")
            for j in range(self.ngroups, n):
                self.run_group(j)
            c.check()
            return
        for j in range(n):
            self.run_group(j)
        c.check()
        n0 = int(self.d_size[0].item())
        pay0 = bytes(self.d_pay[0, :n0].cpu().numpy())
        self.payload0 = n0
        if self.q == 50 and sha(pay0) != BIG_RECOMPRESSED_SHA:
            raise SystemExit("compressed stream differs from the pinned reference bytes")
        for f in range(self.per_step):
            nk = int(self.d_size[f].item())
            if bytes(self.d_pay[f, :nk].cpu().numpy()) != pay0:
                raise SystemExit(f"frame slot {f}: compressed stream differs from slot 0's")
        self.want_decode = None
        if isinstance(c, GpuCodec):
            want = self.want_decode = c.codecs[0].decompress(pay0, self.w, self.h, self.q3)
            for k in range(self.nf):
                for b in range(self.B):
                    if bytes(self.d_out[k, b * self.samples:(b + 1) * self.samples].cpu().numpy()) != want:
                        raise SystemExit(f"context {k} frame {b}: device round trip differs from the host-API decode")
        self.verified["first_pass"] = (f"{self.per_step} streams == the pinned reference bytes "
                                       f"{BIG_RECOMPRESSED_SHA[:8]}; every round trip == the host-API decode")

    def timed(self, steps, dist, dev, gather_chunk):
        """K steps; at N > 1 the streams go to rank 0 (batch.ChunkedGather,
        chunks of about gather_chunk frames, each posted when its launch groups'
        events fire).  Returns (seconds, gathered streams on rank 0 or None);
        self.timing holds this rank's wall / compute / gather-tail seconds and
        gathered bytes, self.gather_bad the ranks whose sizes passed a slot."""
        c = self.codec
        # every output the timed region checks afterwards (verify_timed) is
        # cleared first, so nothing the untimed pass wrote can pass for it
        self.d_pay.zero_()
        self.d_size.zero_()
        self.d_out.zero_()
        gat = None
        if self.world > 1:
            import batch
            gat = batch.ChunkedGather(dist, self.world, self.rank, dev, cap=self.cap)
            dist.barrier()
        c.sync()
        if isinstance(c, CpuCodec):
            c.phase = "timed"
        ev0 = c.marker()
        t0 = time.perf_counter()
        ngr = steps * self.ngroups
        evs, c0, nfr = [], 0, 0
        for j in range(ngr):
            k, nb, slot = self.run_group(j)
            if gat is not None:
                ev = c.event(k)
                if ev is not None:
                    evs.append(ev)
                nfr += nb
                if nfr >= gather_chunk or j == ngr - 1:
                    i1 = slot + nb
                    gat.add(list(range(c0, i1)), [self.d_pay[i] for i in range(c0, i1)], self.d_size[c0:i1], evs)
                    evs, c0, nfr = [], i1, 0
        c.join()
        ev1 = c.marker()
        t_host = time.perf_counter() - t0
        got = gat.finish(steps * self.n_local) if gat is not None else None
        c.sync()
        wall = time.perf_counter() - t0
        compute = ev0.elapsed_time(ev1) / 1e3 if ev0 is not None else t_host
        self.timing = {"wall_s": wall, "compute_s": compute, "gather_tail_s": max(0.0, wall - compute),
                       "gather_bytes": gat.bytes if gat is not None else 0}
        self.gather_bad = sorted(gat.bad_ranks) if gat is not None else []
        if self.world > 1:
            dist.barrier()
        return wall, got

    def verify_timed(self, steps):
        """After the timed region: the streams of its last step and the frames
        its last decode launches wrote (each context's last launch group),
        against the pinned bytes / manifest and the host-API decode."""
        c = self.codec
        c.sync()
        js = range((steps - 1) * self.ngroups, steps * self.ngroups)
        nstream = ndec = 0
        for j in js:
            k, _, nb, slot = self.group_desc(j)
            sizes = self.d_size[slot:slot + nb].cpu().tolist()
            for b in range(nb):
                pay = bytes(self.d_pay[slot + b, :sizes[b]].cpu().numpy())
                if self.name == "batch4k":
                    m = self.manifest[self.gframes[j % self.ngroups * self.B + b]]
                    ok = len(pay) == m["payload_size"] and sha(pay) == m["payload_sha"]
                else:
                    ok = len(pay) == self.payload0 and (sha(pay) == BIG_RECOMPRESSED_SHA if self.q == 50 else True)
                if not ok:
                    raise SystemExit(f"timed region: stream of launch group {j} frame {b} is wrong")
                nstream += 1
        last = {}
        for j in js:  # each context's last launch group decoded into d_out[k]
            last[self.group_desc(j)[0]] = j
        for k, j in sorted(last.items()):
            _, _, nb, _ = self.group_desc(j)
            decs = hashes(self.d_out[k], nb, self.samples)
            for b in range(nb):
                if self.name == "batch4k":
                    want = self.manifest[self.gframes[j % self.ngroups * self.B + b]]["decoded_sha"]
                elif self.want_decode is not None:
                    want = sha(self.want_decode)
                else:
                    continue
                if decs[b] != want:
                    raise SystemExit(f"timed region: decode of launch group {j} frame {b} is wrong")
                ndec += 1
        src = "tests/golden/batch4k_512.json" if self.name == "batch4k" else (
            f"the pinned reference bytes {BIG_RECOMPRESSED_SHA[:8]}" if self.q == 50 else "the first pass's size")
        self.verified["timed_region"] = (f"timed-region outputs checked (cleared before it): the last step's "
                                         f"{nstream} streams == {src}; {ndec} frames of each context's last "
                                         f"decode == " + ("the manifest" if self.name == "batch4k"
                                                          else "the host-API decode"))

    def verify_gathered(self, got, steps):
        """Rank 0, N > 1: the gathered streams in global frame order."""
        if got is None or len(got) != self.world * steps * self.n_local or any(t is None for t in got):
            raise SystemExit("gather: streams missing on rank 0")
        if self.name == "batch4k":
            for s in sorted({0, steps - 1}):
                part = got[s * self.n_total:(s + 1) * self.n_total]
                for f, t in enumerate(part):
                    m = self.manifest[f]
                    if t.numel() != m["payload_size"] or sha(bytes(t.cpu().numpy())) != m["payload_sha"]:
                        raise SystemExit(f"gathered step {s} frame {f}: stream differs from the manifest")
            return (f"rank 0 gathered {len(got)} streams; steps {sorted({0, steps - 1})}: all {self.n_total} "
                    f"frames' size + sha256 == tests/golden/batch4k_512.json")
        for i in sorted({0, len(got) // 2, len(got) - 1}):
            if self.q == 50 and sha(bytes(got[i].cpu().numpy())) != BIG_RECOMPRESSED_SHA:
                raise SystemExit(f"gathered stream {i} differs from the pinned reference bytes")
        return (f"rank 0 gathered {len(got)} streams"
                + (f"; first, middle and last == {BIG_RECOMPRESSED_SHA[:8]}" if self.q == 50 else ""))


def load_manifest():
    with open(MANIFEST_4K) as f:
        return json.load(f)


def hashes(t, n, stride=None):
    """sha256 of rows 0..n-1 of a uint8 tensor (or of n stride-byte pieces of a
    flat one), hashed on host threads."""
    from concurrent.futures import ThreadPoolExecutor
    flat = t.reshape(-1)
    stride = stride or t.shape[-1]

    def one(i):
        return sha(flat[i * stride:(i + 1) * stride].cpu().numpy().tobytes())

    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(one, range(n)))


def k1_roofline(stats, samples_per_frame, frames, B, frame_key):
    """K1 from the stamped launches: 3 B per sample x the samples they covered
    / K1's own summed durations.  The exact-path kernel k_fdct_fix (the units
    K1 could not prove, 0.08 % at q50) is reported beside it, not summed: in
    the pipeline it mostly waits for CU slots behind the other launch groups."""
    k1_ms, k1_n = stats.get("fdct_quant", (0.0, 0))
    if not k1_n or not frames:
        return None
    fix_ms, fix_n = stats.get("fdct_fix", (0.0, 0))
    alg_total = 3 * samples_per_frame * frames
    achieved = alg_total / (k1_ms / 1e3) / 1e9
    avg_s = k1_ms / k1_n / 1e3
    traffic = load_traffic(frame_key, B)
    ceil = valu_ceiling_frac(samples_per_frame)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": "fdct_quant",
            "scope": "k_fdct_quant only: the exact path k_fdct_fix (units the fast path cannot prove) is "
                     "excluded here and summed in fix_kernel.frac_with_fix",
            "fix_kernel": {"kernel": "fdct_fix", "avg_launch_us": round(fix_ms / fix_n * 1e3, 2) if fix_n else None,
                           "frac_with_fix": round(alg_total / ((k1_ms + fix_ms) / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
            "algorithmic_bytes_per_launch": alg_total // k1_n, "avg_launch_us": round(avg_s * 1e6, 2),
            "valu_ceiling_frac": ceil,
            "issue_bound": "valu (fp32 butterflies checked against a rigorous error bound, DESIGN.md §4)"}
    if traffic:
        roof["traffic_gbs"] = round(traffic / avg_s / 1e9, 1)
        roof["traffic_frac"] = round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 4)
    return roof


def valu_ceiling_frac(samples_per_frame):
    """The HBM fraction K1's VALU issue alone allows: a 16-block unit (1,024
    samples, 3,072 algorithmic bytes) occupies one SIMD's VALU issue for
    K1_ISSUE_NS_PER_UNIT ns; 1,024 SIMDs."""
    unit_s = K1_ISSUE_NS_PER_UNIT * 1e-9 / 1024  # seconds of the whole chip per unit
    return round(3 * 1024 / unit_s / 1e9 / HBM_PEAK_GBS, 4)


def host_api_rate(codec_mod, raw, w, h, q, iters):
    """The host-buffer C ABI (myyuv_gpu_dct_compress / _decompress: H2D,
    kernels, D2H, one sync per call) on pageable host buffers allocated once,
    time = t_compress + t_decompress, medians."""
    import numpy as np
    c = codec_mod.Codec(0)
    try:
        src = np.frombuffer(raw, np.uint8).copy()
        pay = np.empty(codec_mod.payload_bound(w, h), np.uint8)
        out = np.empty(w * h * 3 // 2, np.uint8)
        pay.fill(0)
        out.fill(0)
        tc, td = [], []
        for i in range(iters + 3):
            t0 = time.perf_counter()
            n = c.compress_into(src, w, h, (q, q, q), pay)
            t1 = time.perf_counter()
            c.decompress_into(pay[:n], w, h, (q, q, q), out)
            t2 = time.perf_counter()
            if i >= 3:
                tc.append(t1 - t0)
                td.append(t2 - t1)
        if q == 50 and sha(pay[:n].tobytes()) != BIG_RECOMPRESSED_SHA:
            raise SystemExit("host API: compressed stream differs from the pinned reference bytes")
        mc, md = statistics.median(tc), statistics.median(td)
        mp = w * h / 1e6
        return {"value": round(mp / (mc + md), 1), "unit": "MP/s", "compress_ms": round(mc * 1e3, 3),
                "decompress_ms": round(md * 1e3, 3), "round_trips": iters,
                "pcie_bytes": int(2 * (w * h * 3 // 2 + n)),
                "api": "myyuv_gpu_dct_compress + myyuv_gpu_dct_decompress, pageable host buffers"}
    finally:
        c.close()


def host_batch_rate(codec_mod, raw, w, h, q, nframes, reps):
    """The pipelined host-buffer batches (myyuv_gpu_dct_compress_batch /
    _decompress_batch: uploads, kernels and downloads of successive chunks
    overlapped on three streams) over nframes copies of the frame in
    pageable host buffers allocated once; time = t_compress + t_decompress
    of the whole batch, median of reps."""
    import ctypes
    import numpy as np
    c = codec_mod.Codec(0)
    L = codec_mod.load()
    try:
        fb = w * h * 3 // 2
        src = np.tile(np.frombuffer(raw, np.uint8), nframes)
        cap = (codec_mod.payload_bound(w, h) + 3) & ~3
        pay = np.zeros(nframes * cap, np.uint8)
        out = np.zeros(nframes * fb, np.uint8)
        sizes = (ctypes.c_uint32 * nframes)()
        qa = np.array([q, q, q], np.uint8)
        bad = ctypes.c_int64(-1)
        u8 = codec_mod._u8
        tc, td = [], []
        for i in range(reps + 1):
            t0 = time.perf_counter()
            rc = L.myyuv_gpu_dct_compress_batch(c._h, u8(src), nframes, w, h, u8(qa), u8(pay), cap, sizes)
            t1 = time.perf_counter()
            if rc:
                raise codec_mod.CodecError(rc)
            rc = L.myyuv_gpu_dct_decompress_batch(c._h, u8(pay), sizes, cap, nframes, w, h, u8(qa), u8(out),
                                                  ctypes.byref(bad))
            t2 = time.perf_counter()
            if rc:
                raise codec_mod.CodecError(rc, bad.value)
            if i >= 1:
                tc.append(t1 - t0)
                td.append(t2 - t1)
        n0 = int(sizes[0])
        if q == 50 and sha(pay[:n0].tobytes()) != BIG_RECOMPRESSED_SHA:
            raise SystemExit("host batch: compressed stream differs from the pinned reference bytes")
        if any(int(sizes[f]) != n0 for f in range(nframes)) or \
                any(sha(pay[f * cap: f * cap + n0].tobytes()) != sha(pay[:n0].tobytes()) for f in (1, nframes - 1)):
            raise SystemExit("host batch: frames of one input differ")
        dec1 = c.decompress(pay[:n0].tobytes(), w, h, (q, q, q))  # the single-frame call
        if out[:fb].tobytes() != dec1 or out[(nframes - 1) * fb:].tobytes() != dec1:
            raise SystemExit("host batch: decoded frames differ from the single-frame decode")
        mc, md = statistics.median(tc), statistics.median(td)
        mp = w * h / 1e6 * nframes
        pcie = nframes * 2 * (fb + n0)
        return {"value": round(mp / (mc + md), 1), "unit": "MP/s", "frames": nframes,
                "compress_ms": round(mc * 1e3, 3), "decompress_ms": round(md * 1e3, 3), "reps": reps,
                "pcie_bytes": pcie, "pcie_gbs": round(pcie / (mc + md) / 1e9, 2),
                "api": "myyuv_gpu_dct_compress_batch + myyuv_gpu_dct_decompress_batch (pipelined), "
                       "pageable host buffers"}
    finally:
        c.close()


def main(argv=None):
    args = parse(argv)
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)
    if args.launch_selftest:
        launch_selftest()
        return
    import torch
    import myyuv_file

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    name = args.workload if args.workload != "auto" else "chef-big"
    dist = None
    # launch shape (4 x 32 since round 6; 4 x 24 before): the launch groups' overflow lists (~200k blocks) take the CAP-16 tier
    # (round 3: 3 x 24 264.2k against 233.1k MP/s for 4 x 8, flat from 3 x 24 to 3 x 48,
    # profiles/r3zzf_*, r3zzg_*); with round 4's K1, 4 x 24 288.1k / 292.2k against 3 x 24
    # 282.6k / 287.0k at 20 / 40 steps, 5 streams slower (one per hardware queue: 4),
    # profiles/r4j_launch_shapes.txt; round 6 (with K2's ovf class): 4 x 32 356.3k / 357.1k against
    # 4 x 24 351.0k / 352.6k, 4 x 40 354.6k, 4 x 48 354.0k, 3 x 32 351.5k (profiles/r6ac_*, r6ad_*)
    nf = max(1, args.inflight or 4)
    prios = [int(v) for v in args.stream_priority.split(",")] if args.stream_priority else [0]
    big = myyuv_file.YUVFile.load(GOLDEN_BIG)
    if args.cpu_codec:
        dev = torch.device("cpu")
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        from oracle import oracle as O
        codec = CpuCodec(nf, args.cpu_codec_fail, rank)
        raw = O.decompress(big.data, big.width, big.height, tuple(big.params))
    else:
        import myyuv_hip
        if world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        codec = GpuCodec(dev, nf, prios)
        raw = codec.codecs[0].decompress(big.data, big.width, big.height, tuple(big.params))
    if sha(big.decompressed(raw).dumps()) != BIG_DECODED_SHA:
        raise SystemExit("decoded chef-big frame does not match its pinned sha")

    run = Run(name, codec, raw, big, args, world, rank)
    run.alloc_slots(args.steps, args.warmup)
    checked(run.warmup, "the untimed pass", dist, world, rank, dev, args.warmup)

    # ---- timed region: K1 (the roofline kernel) event-stamped on every launch
    # group (the average is over the launches a rocprofv3 kernel trace of this
    # run averages), or on launch group 0 only (--events-ctx0)
    gpu = isinstance(codec, GpuCodec)
    stamped = []
    if gpu and not args.no_kernel_events:
        stamped = codec.codecs[:1] if args.events_ctx0 else codec.codecs
        for c in stamped:
            c.profile(True, kernels=["fdct_quant", "fdct_fix"])
    t, got = run.timed(args.steps, dist, dev, args.gather_chunk)
    checked(codec.check, "the timed region", dist, world, rank, dev, bad_ranks=run.gather_bad)
    checked(run.verify_timed, "the timed region's outputs", dist, world, rank, dev, args.steps)
    stats = {}
    for c in stamped:
        for kname, (kms, kn) in c.kernel_stats().items():
            a, n = stats.get(kname, (0.0, 0))
            stats[kname] = (a + kms, n + kn)
        c.profile(False)
    stamped_frames = args.steps * run.per_step if (stamped and not args.events_ctx0) else 0
    if stamped and args.events_ctx0:
        stamped_frames = sum(run.group_desc(j)[2] for j in range(args.steps * run.ngroups)
                             if run.group_desc(j)[0] == 0)
    ranks = None
    if world > 1:
        ranks = rank_timings(dist, world, dev, run.timing)
        t = max(r["wall_s"] for r in ranks)
        if rank == 0:
            run.verified["gathered"] = run.verify_gathered(got, args.steps)
    # per-kernel breakdown (all kernels stamped, one launch group at a time on
    # context 0), outside the timed region
    breakdown = {}
    if gpu and args.breakdown_steps > 0:
        c0 = codec.codecs[0]
        c0.profile(True)
        for i in range(args.breakdown_steps):
            run.run_group(i % run.ngroups, ctx=0)
        c0.sync_status(codec.sps[0])
        breakdown = c0.kernel_stats()
        c0.profile(False)
    side = None
    b4 = None
    if gpu and not args.no_side and name == "chef-big" and run.q == 50:
        # configs[3]/[4] on every rank (all ranks take part in its gather),
        # before rank 0's own side work so no rank waits in a collective for it
        b4 = batch4k_side(args, codec, raw, big, world, rank, dist, dev)
    if gpu and rank == 0 and not args.no_side:
        side = side_measurements(args, run, codec, raw, big, world, dev)
        if b4 is not None:
            side["batch4k"] = b4

    if rank == 0:
        frames_all = world * args.steps * run.per_step
        value = frames_all * run.mp / t
        frame_key = f"{run.w}x{run.h}"
        roof = k1_roofline(stats, run.samples, stamped_frames, run.B, frame_key)
        kernel_us = {k: round(kms / kn * 1e3, 2) for k, (kms, kn) in breakdown.items() if kn}
        # the same K1 figure with one launch group at a time (the untimed
        # breakdown pass): the kernel alone on the GPU, no co-running group
        roof_iso = None
        if roof and kernel_us.get("fdct_quant"):
            k1_us = kernel_us["fdct_quant"]
            a_iso = 3 * run.samples * run.B / (k1_us * 1e-6) / 1e9
            fix_us = kernel_us.get("fdct_fix") or 0.0
            a_fix = 3 * run.samples * run.B / ((k1_us + fix_us) * 1e-6) / 1e9
            roof_iso = {"kernel": "fdct_quant", "achieved": round(a_iso, 1), "frac": round(a_iso / HBM_PEAK_GBS, 4),
                        "scope": "k_fdct_quant only; frac_with_fix sums the exact path k_fdct_fix",
                        "avg_launch_us": round(k1_us, 2), "fix_avg_us": kernel_us.get("fdct_fix"),
                        "frac_with_fix": round(a_fix / HBM_PEAK_GBS, 4)}
        # the fused decoder (default; K5 + K6 in one kernel, the "huff_decode"
        # id): stream bytes in + 1 B per sample out
        roof_dec = None
        if kernel_us.get("huff_decode") and name == "chef-big":
            alg_d = (run.payload0 + run.samples) * run.B
            ad = alg_d / (kernel_us["huff_decode"] * 1e-6) / 1e9
            roof_dec = {"kernel": "decode_idct (fused K5+K6)", "achieved": round(ad, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ad / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": alg_d,
                        "avg_launch_us": kernel_us["huff_decode"]}
        for k, us in kernel_us.items():
            log(f"kernel {k:16s} {us:9.2f} us/launch")
        cpu = None
        if gpu and world == 1 and args.cpu_seconds > 0:
            crow = raw if name == "chef-big" else bytes(run.d_in[0].cpu().numpy())
            cpu = cpu_baseline(crow, run.w, run.h, run.q, args.cpu_seconds, args.cpu_threads)
        if name == "chef-big":
            workload = (f"chef-with-trumpet-big 4032x3008 IYUV DCT q={run.q} compress+decompress, HBM-resident, "
                        f"{run.per_step} frames/step/GPU (BASELINE configs[1])")
            data = ("chef-with-trumpet-big-DCT-50.myyuv decoded (4032x3008 IYUV, sha-pinned); stand-in for the "
                    f"missing raw 4K; {run.nin} distinct HBM copies")
        else:
            workload = (f"batch of {run.n_total} synthetic 3840x2160 IYUV frames, DCT q={run.q} "
                        f"compress+decompress, dealt round-robin over {world} GPU(s), "
                        f"{'streams gathered to rank 0 over RCCL, ' if world > 1 else ''}"
                        f"HBM-resident (BASELINE configs[3]/[4])")
            data = "synthetic: tiled chef-big decode, per-frame origin (8f mod 4032, 8f mod 3008), SURVEY §8d"
        line = {
            "metric": "megapixels/sec DCT compress+decompress, 4K IYUV; achieved HBM GB/s vs peak",
            "value": round(value, 2), "unit": "MP/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": run.scaling, "vs_baseline": None, "dtype": "u8/int16 (fp32 transform)",
            "data": data,
            "config": {"workload": workload, "frame": f"{run.w}x{run.h}", "quality": run.q,
                       "parallelism": f"frames sharded, dp{world}", "frames_per_step": world * run.per_step,
                       "frames_per_step_per_gpu": run.per_step, "launch_groups_in_flight": nf,
                       "frames_per_launch": run.B, "payload_slot_bytes": run.cap,
                       **({"input_copies": run.nin, "payload_bytes": run.payload0} if name == "chef-big" else {})},
            "verified": run.verified,
            **({"ranks": ranks, "gather": {
                "bytes_to_rank0": sum(r["gather_bytes"] for r in ranks[1:]),
                "ingress_gbs": round(sum(r["gather_bytes"] for r in ranks[1:]) / t / 1e9, 2),
                "max_gather_tail_s": round(max(r["gather_tail_s"] for r in ranks), 6)}} if ranks else {}),
            "roofline": roof, "roofline_isolated": roof_iso, "roofline_decode_isolated": roof_dec,
            "cpu_baseline": cpu,
            "kernel_us": kernel_us or None,
            "side": side,
        }
        if args.cpu_codec:
            line["codec"] = "cpu restatement (oracle/, --cpu-codec: a test of the loop, not a measurement)"
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.destroy_process_group()


def side_measurements(args, run, codec, raw, big, world, dev):
    """Rank 0, outside the timed region (SURVEY.md §8f rows 1 and 3, §8d's
    end-to-end API rate, and configs[3] at N = 1)."""
    import torch
    import myyuv_hip
    side = {}
    # decode-only batched rate: the same launch groups, decompress only, from
    # the streams the timed region left in HBM
    nd = args.steps * run.ngroups
    for j in range(run.nf):
        run.decode_group(j)
    codec.sync()
    t0 = time.perf_counter()
    for j in range(nd):
        run.decode_group(j)
    codec.join()
    codec.sync()
    td = time.perf_counter() - t0
    codec.check()
    side["decode_only"] = {"value": round(args.steps * run.per_step * run.mp / td, 2), "unit": "MP/s",
                           "frames": args.steps * run.per_step}
    # K7 BMP -> IYUV on a 4032x3008 BGRA bottom-up frame: 4 B in + 1.5 B out
    # per pixel, streaming, so its bound is HBM
    w, h = big.width, big.height
    c0, sp0 = codec.codecs[0], codec.sps[0]
    bgra = torch.randint(0, 256, (w * h * 4,), dtype=torch.uint8, device=dev)
    d_iy = torch.empty(w * h * 3 // 2, dtype=torch.uint8, device=dev)
    for _ in range(3):
        c0.bmp_to_iyuv_device(bgra.data_ptr(), w, h, 32, d_iy.data_ptr(), sp0)
    c0.sync_status(sp0)
    c0.profile(True, kernels=["bmp_to_iyuv"])
    for _ in range(50):
        c0.bmp_to_iyuv_device(bgra.data_ptr(), w, h, 32, d_iy.data_ptr(), sp0)
    c0.sync_status(sp0)
    kms, kn = c0.kernel_stats()["bmp_to_iyuv"]
    c0.profile(False)
    if kn:
        alg = w * h * 4 + w * h * 3 // 2
        a7 = alg / (kms / kn * 1e-3) / 1e9
        side["bmp_to_iyuv"] = {"bound": "hbm", "achieved": round(a7, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(a7 / HBM_PEAK_GBS, 4),
                               "algorithmic_bytes_per_launch": alg,
                               "avg_launch_us": round(kms / kn * 1e3, 2), "frame": f"{w}x{h} BGRA"}
    del bgra, d_iy
    if args.host_api_iters > 0:
        side["host_api"] = host_api_rate(myyuv_hip, raw, w, h, run.q, args.host_api_iters)
    if args.host_batch_frames > 0:
        side["host_batch"] = host_batch_rate(myyuv_hip, raw, w, h, run.q, args.host_batch_frames, 5)
    return side


def batch4k_side(args, codec, raw, big, world, rank, dist, dev):
    """configs[3]/[4] after the timed region, on every rank: the 512-frame
    batch dealt round-robin over the ranks (every stream and decode of the
    first pass checked against the manifest on the rank that made it), then
    timed passes with the streams gathered to rank 0 at N > 1 (rank 0 checks
    the gathered streams of the first and last pass).  Strong scaling: the
    same batch at every N, so these values form that workload's curve."""
    import torch
    a = parse(["--workload", "batch4k", "--frames", str(args.frames), "--inflight", str(args.inflight),
               "--gather-chunk", str(args.gather_chunk)])
    run = Run("batch4k", codec, raw, big, a, world, rank)
    passes = 3
    run.alloc_slots(passes, 1)
    checked(run.warmup, "side.batch4k's untimed pass", dist, world, rank, dev, 1)
    t, got = run.timed(passes, dist, dev, a.gather_chunk)
    checked(codec.check, "side.batch4k's timed passes", dist, world, rank, dev, bad_ranks=run.gather_bad)
    checked(run.verify_timed, "side.batch4k's timed outputs", dist, world, rank, dev, passes)
    out = None
    if world > 1:
        ranks = rank_timings(dist, world, dev, run.timing)
        t = max(r["wall_s"] for r in ranks)
    if rank == 0:
        out = {"value": round(passes * run.n_total * run.mp / t, 2), "unit": "MP/s", "n_gpus": world,
               "scaling": "strong", "frames": run.n_total, "passes": passes,
               "ms_per_pass": round(t / passes * 1e3, 3), "frames_per_launch": run.B,
               "verified": run.verified["first_pass"], "verified_timed": run.verified["timed_region"]}
        if world > 1:
            out["verified_gathered"] = run.verify_gathered(got, passes)
            out["max_gather_tail_s"] = round(max(r["gather_tail_s"] for r in ranks), 6)
    del run, got
    torch.cuda.empty_cache()
    return out


def checked(fn, what, dist, world, rank, dev, *a, bad_ranks=()):
    """Runs fn(*a) (a codec check or the untimed pass); at N > 1 every rank's
    outcome is all-gathered, and if any rank failed (or reported a payload
    size past its slot, `bad_ranks`), every rank exits non-zero naming them."""
    err = None
    try:
        fn(*a)
    except (SystemExit, Exception) as e:  # noqa: BLE001 — reported to every rank below
        err = str(e) or type(e).__name__
    if world <= 1:
        if err:
            raise SystemExit(err)
        return
    import batch
    codes = batch.agree_status(dist, 1 if err else 0, dev)
    failed = sorted({r for r, c in enumerate(codes) if c} | set(bad_ranks))
    if failed:
        if err:
            log(f"rank {rank}: {err}")
        raise SystemExit(f"bench.py: rank(s) {failed} failed in {what}"
                         + (f" (rank {rank}: {err})" if err else ""))


def rank_timings(dist, world, dev, timing):
    """Every rank's timing record (Run.timing) on every rank, in rank order."""
    import torch
    keys = ("wall_s", "compute_s", "gather_tail_s", "gather_bytes")
    t = torch.tensor([float(timing[k]) for k in keys], dtype=torch.float64, device=dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    out = []
    for r, p in enumerate(parts):
        v = p.cpu().tolist()
        out.append({"rank": r, "wall_s": round(v[0], 6), "compute_s": round(v[1], 6),
                    "gather_tail_s": round(v[2], 6), "gather_bytes": int(v[3])})
    return out


if __name__ == "__main__":
    main()
