"""TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's cpu_baseline): a numpy restatement of
the reference's Sparse-DETR decoder-attention-map helpers (utils/dam.py), the checker for the
HIP ``msda_hip_dam_flat_grid`` kernel.  Never imported by the product path.

attn_map_to_flat_grid (utils/dam.py:20-73), per (batch, layer, head) row of S = sum_l T_l:
for every query q, level l, point p with location x = loc * T_l (no half-pixel shift here,
unlike the sampling itself) and weight a:
    i0 = floor(x), i1 = i0 + 1
    row[start_l + i0] += a * (x - i1)      # the reference's "margin_end": <= 0
    row[start_l + i1] += a * (x - i0)
each only when 0 <= i < T_l (an out-of-range tap adds 0 at index 0 in the reference).
"""
import numpy as np

__all__ = ["attn_map_to_flat_grid", "idx_to_flat_grid", "compute_corr"]


def attn_map_to_flat_grid(temporal_shapes, level_start_index, sampling_locations, attention_weights):
    """sampling_locations (B, NL, Lq, M, L, P[, 1]), attention_weights (B, NL, Lq, M, L, P)
    -> (B, NL, M, S) float32 (utils/dam.py:20-73)."""
    loc = np.asarray(sampling_locations, dtype=np.float32)
    if loc.ndim == 7:
        loc = loc[..., 0]
    aw = np.asarray(attention_weights, dtype=np.float32)
    shapes = [int(t) for t in np.asarray(temporal_shapes).reshape(-1)]
    starts = [int(s) for s in np.asarray(level_start_index).reshape(-1)]
    B, NL, Lq, M, L, P = aw.shape
    S = sum(shapes)
    out = np.zeros((B * NL * M, S), dtype=np.float32)
    for l, (T, st) in enumerate(zip(shapes, starts)):
        # (B, NL, M, Lq * P): the reference's permute(0, 1, 3, 2, 5, 4) row order
        x = (loc[:, :, :, :, l, :] * np.float32(T)).transpose(0, 1, 3, 2, 4).reshape(B * NL * M, -1)
        a = aw[:, :, :, :, l, :].transpose(0, 1, 3, 2, 4).reshape(B * NL * M, -1)
        i0 = np.floor(x).astype(np.int64)
        i1 = i0 + 1
        m_start = (x - i0.astype(np.float32)).astype(np.float32)      # >= 0
        m_end = (x - i1.astype(np.float32)).astype(np.float32)        # <= 0
        for tid, margin in ((i0, m_end), (i1, m_start)):
            valid = (tid >= 0) & (tid < T)
            w = (a * valid * margin).astype(np.float32)
            idx = np.where(valid, tid + st, 0)
            for r in range(out.shape[0]):
                np.add.at(out[r], idx[r], w[r])
    return out.reshape(B, NL, M, S)


def idx_to_flat_grid(temporal_shapes, idx):
    """utils/dam.py:12-17: one-hot rows of the selected token indices."""
    idx = np.asarray(idx, dtype=np.int64)
    S = int(np.sum(np.asarray(temporal_shapes)))
    grid = np.zeros((idx.shape[0], S), dtype=np.float32)
    for r in range(idx.shape[0]):
        grid[r, idx[r]] = 1.0
    return grid


def compute_corr(flat_grid_topk, flat_grid_attn_map, temporal_shapes):
    """utils/dam.py:76-93: overall and per-level fraction of attention mass on the top-k tokens."""
    a = np.atleast_2d(np.asarray(flat_grid_topk, dtype=np.float32))
    m = np.atleast_2d(np.asarray(flat_grid_attn_map, dtype=np.float32))
    corr = [(a * m).sum(-1) / m.sum(-1)]
    start = 0
    for T in np.asarray(temporal_shapes).reshape(-1):
        sl = slice(int(start), int(start + T))
        corr.append((a[:, sl] * m[:, sl]).sum(-1) / m[:, sl].sum(-1))
        start += int(T)
    return corr
