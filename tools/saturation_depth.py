"""How deep into its list each tile saturates (tooling): for the bench's frame
alone (C2 view 0, t_min 1e-4), per tile and per 16x4 slice, the number of
list records composited front to back before every pixel of the slice has
T < t_min (the compositor's early termination), from the frame's own records
and tile lists (gsr_debug_copy), evaluated with the compositor's interval
form in torch (float32; statistics, not parity).  Beside it, the depth a
conservative bound reaches: per record and slice, the alpha at the slice's
four corner pixels (alpha = opacity * 2^pw with pw concave, so its minimum over
the slice is at a corner) counts when the record's rectangle and keep interval
cover the whole slice; the slice is known saturated once the product of
(1 - 0.99 min-alpha) falls below t_min / 2, and with 192-record chunks every
chunk after that one could skip the slice ("bound_*" keys).
usage (GPU box): python tools/saturation_depth.py [out.json]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gsviewer_amd.gaussian_data import garden_standin  # noqa: E402
from gsviewer_amd.multiview import view_of  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into  # noqa: E402
from helpers import grab_debug  # noqa: E402

T_MIN = 1e-4


def main():
    H, W = 1080, 1920
    g = garden_standin(1_000_000, seed=1)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    st = RenderSettings(t_min=T_MIN, out_layout=1)
    render_into(ctx, scene, camera_from(view_of(0, H, W)), st, out)
    torch.cuda.synchronize()
    d = grab_debug(ctx, ctx.stats())
    recs = torch.from_numpy(d["records"].view(np.float32).reshape(-1, 12).copy()).cuda()
    u32 = torch.from_numpy(d["records"].view(np.uint32).reshape(-1, 12).astype(np.int64)).cuda()
    lst = torch.from_numpy(d["tile_list"].astype(np.int64)).cuda()
    ranges = d["ranges"].astype(np.int64)
    tiles_x = (W + 15) // 16
    lane = torch.arange(64, device="cuda")
    col = lane % 16
    row = lane // 16
    depth_tile, slice_depths, slice_work, lens = [], [], [], []
    bound_depths, bound_chunk_work, chunk, all_touch = [], [], 192, []
    for t in range(len(ranges)):
        b, e = ranges[t]
        L = int(e - b)
        lens.append(L)
        if L == 0:
            depth_tile.append(0)
            continue
        ids = lst[b:e]
        r = recs[ids]
        cx, cy, s, qa, qb, qc, cr, mid = r[:, 0], r[:, 1], r[:, 2], r[:, 4], r[:, 5], r[:, 6], r[:, 8], r[:, 11]
        xs, ys = u32[ids, 3], u32[ids, 7]
        x0, x1, r0, r1 = xs & 0xFFFF, xs >> 16, ys & 0xFFFF, ys >> 16
        tx, ty = t % tiles_x, t // tiles_x
        worst = 0
        for k in range(4):  # 16x4 slices
            px_x = tx * 16 + col
            px_row = ty * 16 + 4 * k + row
            px = px_x.float() + 0.5
            pyw = (H - 1 - px_row).float() + 0.5
            dx = px[None, :] - cx[:, None]
            dy = pyw[None, :] - cy[:, None]
            pw = (qa[:, None] * dx * dx + qb[:, None] * dx * dy + qc[:, None] * dy * dy) - mid[:, None]
            keep = pw.abs() <= -mid[:, None]
            cov = ((px_x[None, :] >= x0[:, None]) & (px_x[None, :] <= x1[:, None]) &
                   (px_row[None, :] >= r0[:, None]) & (px_row[None, :] <= r1[:, None]) & (px_row[None, :] < H) &
                   (px_x[None, :] < W))
            a1 = (s[:, None] * torch.exp2(pw)).clamp(0, 1)
            alpha = torch.where(keep & cov, 0.99 * a1, torch.zeros_like(a1))
            T = torch.cumprod(1 - alpha, dim=0)
            live_px = (px_row < H) & (px_x < W)
            sat = (T < T_MIN) | ~live_px[None, :]
            full = sat.all(dim=1)
            idx = int(torch.nonzero(full)[0]) + 1 if bool(full.any()) else L
            touch = cov.any(dim=1)
            # conservative bound from the slice's corner pixels
            live_rows = px_row[::16][(px_row[::16] < H)]
            cx0, cx1 = tx * 16, min(tx * 16 + 15, W - 1)
            rr0, rr1 = int(live_rows.min()), int(live_rows.max())
            full = (x0 <= cx0) & (x1 >= cx1) & (r0 <= rr0) & (r1 >= rr1)
            amin = torch.full_like(s, 1.0)
            okc = full.clone()
            for ccx in (cx0, cx1):
                for ccr in (rr0, rr1):
                    ddx = (ccx + 0.5) - cx
                    ddy = (H - 1 - ccr + 0.5) - cy
                    pwc = qa * ddx * ddx + qb * ddx * ddy + qc * ddy * ddy - mid
                    okc &= pwc.abs() <= -mid * 0.999
                    amin = torch.minimum(amin, (s * torch.exp2(pwc)).clamp(0, 1))
            ab = torch.where(okc, 0.99 * amin * (1 - 1e-5), torch.zeros_like(amin))
            Tb = torch.cumprod((1 - ab).double(), dim=0)
            hit = torch.nonzero(Tb < T_MIN / 2)
            bidx = int(hit[0]) + 1 if len(hit) else L
            bound_depths.append(bidx)
            # chunks up to and including the one holding record bidx - 1 composite the slice
            last_chunk = (bidx - 1) // chunk
            bound_chunk_work.append(int(touch[:min(L, (last_chunk + 1) * chunk)].sum()))
            slice_depths.append(idx)
            slice_work.append(int(touch[:idx].sum()))
            all_touch.append(int(touch.sum()))
            worst = max(worst, idx)
        depth_tile.append(worst)
    lens = np.array(lens)
    dt = np.array(depth_tile)
    deep = lens > 192
    res = {
        "instances": int(lens.sum()),
        "tile_len": {"max": int(lens.max()), "p99": float(np.percentile(lens, 99)), "mean": float(lens.mean())},
        "saturation_depth_records": {"max": int(dt.max()), "p99": float(np.percentile(dt, 99)),
                                     "p90": float(np.percentile(dt, 90)), "mean": float(dt.mean())},
        "tiles_deeper_than_192": int(deep.sum()),
        "records_until_tile_saturation": int(dt.sum()),
        "fraction_of_instances": float(dt.sum() / lens.sum()),
        "slice_walk_records": int(np.sum(slice_work)),
        "slice_walk_fraction": float(np.sum(slice_work) / lens.sum()),
        "all_slice_evaluations": int(sum(int(x) for x in all_touch)),
        "bound_depth_sum": int(np.sum(bound_depths)),
        "bound_vs_exact_depth": float(np.sum(bound_depths) / max(1, np.sum(slice_depths))),
        "bound_chunk_slice_evaluations": int(np.sum(bound_chunk_work)),
        "bound_chunk_fraction_of_evaluations": float(np.sum(bound_chunk_work) / max(1, sum(all_touch))),
        "deep_tiles_depth_hist": np.histogram(dt[deep], bins=[0, 192, 384, 768, 1536, 3072, 6144, 12288, 1 << 20])[0]
        .tolist(),
    }
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)
        np.savez(os.path.splitext(sys.argv[1])[0] + "_tiles.npz", tile_len=lens, tile_depth=dt,
                 slice_depth=np.array(slice_depths), slice_work=np.array(slice_work))


if __name__ == "__main__":
    main()
