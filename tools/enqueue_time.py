"""Diagnostic: host time to enqueue the bench's launch groups (3 contexts x
4-frame batches, compress + decompress) against the GPU time they take —
whether launch overhead (and so HIP graphs) could matter."""
import os, sys, time
ROOT='/root/repo' if os.path.exists('/root/repo/bench.py') else os.getcwd()
sys.path[:0]=[ROOT, os.path.join(ROOT,'yuv-manipulations-2_amd')]
import torch, myyuv_file, myyuv_hip
NF,B,G=3,4,120
g=myyuv_file.YUVFile.load(os.path.join(ROOT,'tests/golden/chef-with-trumpet-big-DCT-50.myyuv'))
w,h=g.width,g.height
cs=[myyuv_hip.Codec(0) for _ in range(NF)]
raw=cs[0].decompress(g.data,w,h,tuple(g.params))
dev=torch.device('cuda',0)
sts=[torch.cuda.current_stream(dev)]+[torch.cuda.Stream(dev) for _ in range(NF-1)]
cap=(myyuv_hip.payload_bound(w,h)+3)&~3; fb=w*h*3//2
d_in=torch.frombuffer(bytearray(raw*B),dtype=torch.uint8).to(dev)
d_out=torch.empty((NF,B*fb),dtype=torch.uint8,device=dev)
d_pay=torch.empty((NF,B*cap),dtype=torch.uint8,device=dev)
d_sz=torch.zeros((NF,B),dtype=torch.int32,device=dev)
for c in cs: c.reserve_batch(w,h,B)
q=(50,50,50)
def grp(j):
    k=j%NF; sp=sts[k].cuda_stream
    cs[k].compress_batch_device(d_in.data_ptr(),B,w,h,q,d_pay[k].data_ptr(),cap,d_sz[k].data_ptr(),sp)
    cs[k].decompress_batch_device(d_pay[k].data_ptr(),d_sz[k].data_ptr(),cap,B,w,h,q,d_out[k].data_ptr(),sp)
for j in range(6): grp(j)
torch.cuda.synchronize()
t0=time.perf_counter()
for j in range(G): grp(j)
t1=time.perf_counter()
torch.cuda.synchronize()
t2=time.perf_counter()
print(f"enqueue {1e3*(t1-t0):.2f} ms, total {1e3*(t2-t0):.2f} ms, per group enqueue {1e6*(t1-t0)/G:.1f} us, MP/s {G*B*w*h/1e6/(t2-t0):.0f}")
