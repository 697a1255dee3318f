import os, sys, time
sys.argv=['bench.py']
ROOT=os.environ.get('GRAFT_REPO_ROOT','/root/repo')
sys.path[:0]=[ROOT, ROOT+'/yuv-manipulations-2_amd']
import torch, myyuv_hip, myyuv_file
g=myyuv_file.YUVFile.load(ROOT+'/tests/golden/chef-with-trumpet-big-DCT-50.myyuv')
w,h=g.width,g.height
cs=[myyuv_hip.Codec(0) for _ in range(3)]
raw=cs[0].decompress(g.data,w,h,tuple(g.params))
dev=torch.device('cuda',0)
sts=[torch.cuda.current_stream(dev)]+[torch.cuda.Stream(dev) for _ in range(2)]
cap=myyuv_hip.payload_bound(w,h)
d_in=torch.frombuffer(bytearray(raw),dtype=torch.uint8).to(dev)
d_out=torch.empty((3,w*h*3//2),dtype=torch.uint8,device=dev)
d_pay=torch.empty((60,cap),dtype=torch.uint8,device=dev); d_size=torch.zeros(60,dtype=torch.int32,device=dev)
for c in cs: c.reserve(w,h)
def step(i):
    k=i%3; c=cs[k]; sp=sts[k].cuda_stream
    c.compress_device(d_in.data_ptr(),w,h,(50,50,50),d_pay[i].data_ptr(),cap,d_size[i:i+1].data_ptr(),sp)
    c.decompress_device(d_pay[i].data_ptr(),d_size[i:i+1].data_ptr(),cap,w,h,(50,50,50),d_out[k].data_ptr(),sp)
for i in range(6): step(i)
torch.cuda.synchronize()
for prof in (False, True):
    for c in cs: c.profile(prof, kernels=["fdct_quant"] if prof else None)
    t0=time.perf_counter()
    for i in range(60): step(i)
    t1=time.perf_counter()
    torch.cuda.synchronize()
    t2=time.perf_counter()
    print(f"profile={prof}: host enqueue {((t1-t0)/60)*1e6:.1f} us/step, wall {((t2-t0)/60)*1e6:.1f} us/step")
    for c in cs: c.sync_status(None)
