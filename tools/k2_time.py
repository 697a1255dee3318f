"""Diagnostic: K2 per-stage wave cycles (stamp build) on the bench frame."""
import ctypes, os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, 'yuv-manipulations-2_amd')]
os.environ.setdefault('MYYUV_HIP_LIB', os.path.join(R, 'yuv-manipulations-2_amd/build/stamps/libmyyuv_hip.so'))
import torch, myyuv_hip, myyuv_file, synth
c = myyuv_hip.Codec(0)
L = myyuv_hip.load()
names = ['', 'stage1', 'sync', 'map', 'heap+len', 'sort', 'emit']
def run(raw, w, h, q, label):
    d_in = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    cap = myyuv_hip.payload_bound(w, h)
    d_pay = torch.empty(cap, dtype=torch.uint8, device='cuda'); d_size = torch.zeros(1, dtype=torch.int32, device='cuda')
    sp = torch.cuda.current_stream().cuda_stream
    for i in range(3):
        c.compress_device(d_in.data_ptr(), w, h, (q,q,q), d_pay.data_ptr(), cap, d_size.data_ptr(), sp)
    c.sync_status(sp)
    st = (ctypes.c_ulonglong * 8)()
    L.myyuv_debug_k2_stamps(st)
    c.profile(True)
    for i in range(10):
        c.compress_device(d_in.data_ptr(), w, h, (q,q,q), d_pay.data_ptr(), cap, d_size.data_ptr(), sp)
    c.sync_status(sp)
    L.myyuv_debug_k2_stamps(st)
    nw = ((w*h*3//2)//64 + 63)//64 * 10
    ks = c.kernel_stats()
    print(label, 'huff_encode us', round(ks['huff_encode'][0]/ks['huff_encode'][1]*1e3,1),
          ' cycles/wave:', {names[k]: round(st[k]/nw) for k in range(1,7)}, flush=True)
g = myyuv_file.YUVFile.load(os.path.join(R, 'tests/golden/chef-with-trumpet-big-DCT-50.myyuv'))
w, h = g.width, g.height
raw = c.decompress(g.data, w, h, (50, 50, 50))
run(raw, w, h, 50, 'chef-big q50')
run(raw, w, h, 90, 'chef-big q90')
run(synth.noise_frame(2048, 1024).tobytes(), 2048, 1024, 50, 'noise q50')
