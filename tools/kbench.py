#!/usr/bin/env python3
"""Diagnostic kernel timing for experimental builds (no correctness checks):
the bench workload (chef-big 4032x3008 q50, HBM-resident) through
compress_device + decompress_device, per-kernel HIP-event times.

  MYYUV_HIP_LIB=<dir>/libmyyuv_hip.so python3 tools/kbench.py [steps] [WxH]

WxH: a tiled synthetic frame of that size (SURVEY.md §8d generator) instead.
KB_Q=90: quality for all three planes (default 50).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "yuv-manipulations-2_amd")
sys.path[:0] = [ROOT, PKG]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    import torch
    import myyuv_file
    import myyuv_hip
    from oracle import oracle as O
    g = myyuv_file.YUVFile.load(os.path.join(ROOT, "tests", "golden", "chef-with-trumpet-big-DCT-50.myyuv"))
    w, h = g.width, g.height
    raw = O.decompress(g.data, w, h, tuple(g.params))
    q = (int(os.environ.get("KB_Q", "50")),) * 3
    if len(sys.argv) > 2:
        import synth
        ws, hs = w, h
        w, h = (int(v) for v in sys.argv[2].split("x"))
        raw = bytes(synth.tiled_frame(raw, ws, hs, w, h))
    expect = O.decompress(O.compress(raw, w, h, q), w, h, q)
    dev = torch.device("cuda", 0)
    codec = myyuv_hip.Codec(0)
    cap = myyuv_hip.payload_bound(w, h)
    st = torch.cuda.Stream(dev)  # explicit: handle 0 would mean the context's own stream
    sp = st.cuda_stream
    torch.cuda.set_stream(st)
    d_in = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    d_out = torch.empty(w * h * 3 // 2, dtype=torch.uint8, device=dev)
    d_pay = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_size = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.reserve(w, h)
    rc = None
    for it in range(2):
        codec.profile(it == 1)
        for _ in range(steps if it else 3):
            codec.compress_device(d_in.data_ptr(), w, h, q, d_pay.data_ptr(), cap, d_size.data_ptr(), sp)
            codec.decompress_device(d_pay.data_ptr(), d_size.data_ptr(), cap, w, h, q, d_out.data_ptr(), sp)
        try:
            rc, bad = codec.sync_status(sp)
        except Exception as e:  # ablation builds may produce invalid streams
            rc = repr(e)
    stats = codec.kernel_stats()
    ok = bytes(d_out.cpu().numpy()) == expect
    # wall time per call on the stream (no per-kernel stamps): compress alone,
    # then the round trip (kernels of one call may run on two streams)
    codec.profile(False)
    walls = []
    for rt in (False, True):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(steps):
            codec.compress_device(d_in.data_ptr(), w, h, q, d_pay.data_ptr(), cap, d_size.data_ptr(), sp)
            if rt:
                codec.decompress_device(d_pay.data_ptr(), d_size.data_ptr(), cap, w, h, q, d_out.data_ptr(), sp)
        t1.record()
        torch.cuda.synchronize()
        walls.append(t0.elapsed_time(t1) / steps * 1e3)
    print(f"{os.environ.get('MYYUV_HIP_LIB', 'default')} {w}x{h} q{q[0]}: rc={rc} roundtrip_equal={ok}")
    for k, (ms, n) in stats.items():
        if n:
            print(f"  {k:14s} {ms / n * 1e3:9.2f} us")
    print(f"  compress wall    {walls[0]:9.2f} us")
    print(f"  round trip wall  {walls[1]:9.2f} us")
    codec.close()


if __name__ == "__main__":
    main()
