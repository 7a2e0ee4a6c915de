import sys, numpy as np, time
sys.path.insert(0,'tests'); sys.path.insert(0,'.')
from gsviewer_amd.gaussian_data import garden_standin
from gsviewer_amd.camera import Camera
from oracle import gl_oracle as O
from helpers import uniforms_for
t=time.time()
g = garden_standin(1_000_000, seed=1, sh_degree=0)
cam = Camera(1080, 1920)
U = uniforms_for(cam)
vs = O.vertex_stage(g.flat(), g.sh_dim, U)
x0,x1,r0,r1 = O.splat_rects(vs, U)[:4]
print('vs', time.time()-t)
T=16; tiles_x=(1920+15)//16
ok = vs["visible"] & (x0 <= x1) & (r0 <= r1)
gid = np.nonzero(ok)[0]
tx0, tx1, ty0, ty1 = x0[gid] // T, x1[gid] // T, r0[gid] // T, r1[gid] // T
ntx = tx1 - tx0 + 1; cnt = ntx * (ty1 - ty0 + 1)
rep = np.repeat(np.arange(len(gid)), cnt)
k = np.arange(int(cnt.sum())) - np.repeat(np.cumsum(cnt) - cnt, cnt)
tile = ((ty0[rep] + k // ntx[rep]) * tiles_x + tx0[rep] + k % ntx[rep]).astype(np.int64)
ig = gid[rep]
vis = np.nonzero(vs["visible"])[0]
b = (-vs["view_z"].astype(np.float32)).view(np.uint32).astype(np.uint64)
key = np.where(b & 0x80000000, ~b & 0xFFFFFFFF, b | 0x80000000)
kmin, kmax = int(key[vis].min()), int(key[vis].max())
B=(kmax-kmin).bit_length(); print('instances', len(tile), 'B', B)
for coarse in (16, 18, 20, 22):
    s0=max(0,B-coarse)
    ck=(key[ig]-kmin)>>np.uint64(s0)
    o=np.lexsort((ck, tile)); t2=tile[o]; c2=ck[o]
    # runs of equal (tile, ck)
    same = (t2[1:]==t2[:-1]) & (c2[1:]==c2[:-1])
    starts = np.flatnonzero(np.concatenate([[True], ~same]))
    lens = np.diff(np.concatenate([starts,[len(t2)]]))
    big = lens[lens>1]
    print(coarse, 'runs>1', len(big), 'items in runs', big.sum(), 'max', lens.max(), 'sum L^2', int((big.astype(np.int64)**2).sum()), 'p99', np.percentile(big,99) if len(big) else 0)
