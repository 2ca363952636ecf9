"""TEST INFRASTRUCTURE — CPU restatement of the reference's test-time patch
placements: ``PatchTransformer_test_mode``
(load_data.py:1233-1722) and ``PatchTransformer_vanishing``
(load_data.py:985-1230).  Only tests/ import this.

Follows the reference op for op.  Randomness is explicit:
  test mode: angle [B] (radians) and upick [B] U[0,1) — random.randint(0, N)
             (load_data.py:1682) becomes floor(upick * (N + 1));
  vanishing: contrast/bright [B*n], noise [B*n,3,P,P] U(-1,1), angle [B*n],
             offx/offy [B*n] U(-0.2,0.2) (load_data.py:1052-1101, 1131-1143).

Geometry (theta, affine_grid, grid_sample) of the test mode is evaluated in
float64 and each resampled tensor rounded to fp32, as the HIP path does
(the fp32 affine grid loses ~1e-4 px to cancellation); label
arithmetic, the mask == 1 test and the occupancy map stay in fp32 as in the
reference.  The vanishing transformer is restated in the default dtype, so a
test evaluates it in float64 with torch.set_default_dtype.
Sorting by area uses a stable sort (the reference's torch.sort leaves the
order of equal areas unspecified).
"""
import math

import torch
import torch.nn.functional as F

from .reference_path import median_pool7, NOISE_FACTOR

SCALE_FACTOR = 2.          # load_data.py:32
VANISH_PRE_SCALE = 8.0     # load_data.py:1116


def lab_transform_test(lab_batch_origin):
    """load_data.py:1295-1320 ([B,n,7] -> [B,1,7], fp32)."""
    B = lab_batch_origin.size(0)
    sel = torch.zeros(B, 1, 7, dtype=lab_batch_origin.dtype)
    area = lab_batch_origin[:, :, 2] * lab_batch_origin[:, :, 3]
    max_value, max_index = torch.max(area, 1)
    _, min_index = torch.min(area, 1)
    if len(lab_batch_origin[0]) == 1:
        sel[0, :, :] = 0.25
    else:
        for i in range(B):
            if max_value[i] > 0.99:
                sel[i, :, :] = 0.25
            else:
                sel[i, :, :] = (lab_batch_origin[i, max_index[i], :] + lab_batch_origin[i, min_index[i], :]) / 2.
    return sel, max_index, min_index


def inter_axis_cal(lab_batch, semi_edge, img_size):
    """load_data.py:1322-1430, literally (fp32 map; Python slices of int()
    bounds; the early exit with its temp_lab[0:i-1] sum)."""
    lab_batch = lab_batch.squeeze(0)
    lab_scale = lab_batch * img_size
    lab_area = lab_scale[:, 2] * lab_scale[:, 3]
    _, sorted_index = torch.sort(lab_area, stable=True)
    len_lab = len(lab_batch)
    temp_lab = torch.zeros([len_lab, img_size, img_size])
    k = int(semi_edge)
    temp_lab[:, 0:k, :] = 1
    temp_lab[:, -k:, :] = 1
    temp_lab[:, :, 0:k] = 1
    temp_lab[:, :, -k:] = 1
    for i in range(len_lab):
        sum_lab = torch.sum(temp_lab, dim=0)
        if len(torch.nonzero(sum_lab == 0)) == 0:
            return torch.sum(temp_lab[0:i - 1, :, :], dim=0)
        lab_index = lab_scale[sorted_index[i]]
        cx, cy, W, H = lab_index[0], lab_index[1], lab_index[2], lab_index[3]
        temp_lab[i, int(cx - W / 2 - semi_edge):int(cx + W / 2 + semi_edge),
                 int(cy - H / 2 - semi_edge):int(cy + H / 2 + semi_edge)] = 1
    temp_return = torch.sum(temp_lab, dim=0)
    if len(torch.nonzero(temp_return == 0)) == 0:
        return torch.sum(temp_lab[0:len_lab - 1, :, :], dim=0)
    return temp_return


def free_cells_rule(lab_batch, semi_edge, img_size, return_m=False):
    """The closed form po_place_* implement (csrc/place_ops.hip tm_free): with
    c(p) the first box (area order) covering cell p and M its max over the
    non-border cells, the free cells are the non-border cells with c == M,
    every cell when M == 0 or (M == -1 and n == 1), none when M == -1 and
    n >= 2.  Returns a bool [S,S] map ([x][y]); tests check it against
    inter_axis_cal's zeros."""
    lab = lab_batch.squeeze(0)
    S = img_size
    lab_scale = lab * S
    order = torch.sort(lab_scale[:, 2] * lab_scale[:, 3], stable=True)[1]
    n = len(lab)
    k = int(semi_edge)
    cover = torch.full((S, S), n, dtype=torch.int64)
    for i in reversed(range(n)):
        cx, cy, W, H = lab_scale[order[i]][:4]
        sl_x = slice(int(cx - W / 2 - semi_edge), int(cx + W / 2 + semi_edge))
        sl_y = slice(int(cy - H / 2 - semi_edge), int(cy + H / 2 + semi_edge))
        cover[sl_x, sl_y] = i
    border = torch.ones(S, S, dtype=torch.bool)
    if k > 0:
        border[k:S - k, k:S - k] = False
    inner = cover[~border]
    M = int(inner.max()) if inner.numel() else -1
    if M == 0 or (M == -1 and n == 1):
        free = torch.ones(S, S, dtype=torch.bool)
    elif M < 0:
        free = torch.zeros(S, S, dtype=torch.bool)
    else:
        free = (~border) & (cover == M)
    return (free, M) if return_m else free


def _grid_sample64(x, theta, S):
    grid = F.affine_grid(theta, [x.size(0), x.size(1), S, S], align_corners=False)
    return F.grid_sample(x, grid, align_corners=False)


def test_mode_place(adv_patch, lab_batch, img_size, angle, upick, scale_factor=SCALE_FACTOR, do_rotate=True):
    """PatchTransformer_test_mode.forward (load_data.py:1432-1722) for one
    image: lab_batch [1,n,7], angle / upick python floats (fp32 values).
    -> (adv_patch_mask [1,1,3,S,S] fp32, info dict).  Raises where the
    reference raises."""
    S = img_size
    mp = median_pool7(adv_patch.unsqueeze(0))                       # 1451-1452
    P = mp.size(-1)
    pad = (S - P) / 2                                               # 1454
    adv = torch.clamp(mp, 0.0, 1.)                                  # 1490
    msk = torch.ones_like(adv)                                      # 1523
    padl, padr = int(pad + 0.5), int(pad)
    adv = F.pad(adv, (padl, padr, padl, padr), value=0.)            # 1526-1530
    msk = F.pad(msk, (padl, padr, padl, padr), value=0.)
    sel, imax, imin = lab_transform_test(lab_batch)                 # 1578
    n = lab_batch.size(1)
    if n == 1 or float((lab_batch[0, :, 2] * lab_batch[0, :, 3]).max()) > 0.99:   # 1306-1313
        s2 = s3 = 0.25
    else:                                                           # the exact (float64) mean of the two rows
        s2 = (float(lab_batch[0, imax[0], 2]) + float(lab_batch[0, imin[0], 2])) / 2.0
        s3 = (float(lab_batch[0, imax[0], 3]) + float(lab_batch[0, imin[0], 3])) / 2.0
    h2, h3 = s2 * S / scale_factor, s3 * S / scale_factor          # 1582-1596
    target_size = math.sqrt(h2 * h2 + h3 * h3)
    scale = target_size / P                                         # 1605
    a = float(angle) if do_rotate else 0.0
    sn, cs = math.sin(a), math.cos(a)
    theta1 = torch.tensor([[[cs / scale, sn / scale, 0.0], [-sn / scale, cs / scale, 0.0]]],
                          dtype=torch.float64)                      # 1617-1629
    adv1 = _grid_sample64(adv.double(), theta1, S).float()          # 1631-1635
    msk1 = _grid_sample64(msk.double(), theta1, S).float()
    single = msk1[0, 0]                                             # 1644-1650
    ones = torch.nonzero(single == 1)
    if ones.size(0) < 2:
        raise RuntimeError("fewer than two mask==1 pixels")
    rows = ones[:, 0]
    semi_edge = (rows.max() - rows.min()) / 2                       # 1655-1664 (fp32 tensor)
    layout = inter_axis_cal(lab_batch, semi_edge, S)                # 1673
    avail = torch.nonzero(layout == 0)                              # 1678
    N = len(avail)
    pick = min(int(math.floor(float(upick) * (N + 1))), N)          # 1682: randint(0, N), inclusive
    info = {"semi_edge2": int(rows.max() - rows.min()), "n_free": N, "pick": pick,
            "mask_ones": int(ones.size(0))}
    if N == 0:
        raise IndexError("no free position")
    if pick == N:
        raise IndexError("randint drew len(position_available)")
    x, y = int(avail[pick][0]), int(avail[pick][1])                 # 1684-1687
    info.update(x=x, y=y)
    tx = (-x / S + 0.5) * 2                                         # 1689-1690
    ty = (-y / S + 0.5) * 2
    theta2 = torch.tensor([[[1.0, 0.0, tx], [0.0, 1.0, ty]]], dtype=torch.float64)   # 1695-1702
    adv2 = _grid_sample64(adv1.double(), theta2, S).float()         # 1704-1706
    msk2 = _grid_sample64(msk1.double(), theta2, S).float()
    adv2 = torch.clamp(adv2, 0.0, 1.)                               # 1714
    return (adv2 * msk2).unsqueeze(1), info                         # 1715-1722


def vanishing_transformer(adv_patch, lab_batch, img_size, draws, do_rotate=True, rand_loc=False, orient=None,
                          test_real=False):
    """PatchTransformer_vanishing.forward (load_data.py:1021-1230) with
    explicit draws; lab_batch [B,n,5].  -> [B,n,3,S,S]."""
    adv = median_pool7(adv_patch.unsqueeze(0))                      # 1041-1042
    P = adv.size(-1)
    pad = (img_size - P) / 2                                        # 1044
    adv = adv.unsqueeze(0)
    B, n = lab_batch.size(0), lab_batch.size(1)
    adv_batch = adv.expand(B, n, -1, -1, -1)                        # 1047-1048
    contrast = draws["contrast"].view(B, n, 1, 1, 1).expand(-1, -1, 3, P, P)   # 1052-1057
    brightness = draws["bright"].view(B, n, 1, 1, 1).expand(-1, -1, 3, P, P)  # 1060-1065
    noise = draws["noise"].view(B, n, 3, P, P) * NOISE_FACTOR        # 1066-1067
    if not test_real:                                               # 1070-1073
        adv_batch = adv_batch * contrast + brightness + noise
    adv_batch = torch.clamp(adv_batch, 0.0, 1.)                     # 1076
    msk_batch = torch.ones(B, n, 3, P, P, dtype=adv_batch.dtype)    # 1077-1089
    padl, padr = int(pad + 0.5), int(pad)
    adv_batch = F.pad(adv_batch, (padl, padr, padl, padr), value=0.)   # 1090-1094
    msk_batch = F.pad(msk_batch, (padl, padr, padl, padr), value=0.)
    anglesize = B * n
    angle = draws["angle"].clone().view(anglesize) if do_rotate else torch.zeros(anglesize)   # 1095-1101
    lab_scaled = torch.zeros(lab_batch.size())
    for c in range(1, 5):                                           # 1105-1111
        lab_scaled[:, :, c] = lab_batch[:, :, c] * img_size
    pre_scale = VANISH_PRE_SCALE
    target_size = torch.sqrt(((lab_scaled[:, :, 3].mul(1 / pre_scale)) ** 2) +
                             ((lab_scaled[:, :, 4].mul(1 / pre_scale)) ** 2))   # 1119-1120
    target_x = lab_batch[:, :, 1].reshape(anglesize)                # 1122-1126
    target_y = lab_batch[:, :, 2].reshape(anglesize)
    targetoff_x = lab_batch[:, :, 3].reshape(anglesize)
    targetoff_y = lab_batch[:, :, 4].reshape(anglesize)
    if rand_loc:                                                    # 1131-1143
        target_x = target_x + targetoff_x * draws["offx"].view(anglesize)
        target_y = target_y + targetoff_y * draws["offy"].view(anglesize)
    scale = (target_size / P).view(anglesize)                       # 1149-1150
    s = adv_batch.size()
    adv_batch = adv_batch.reshape(s[0] * s[1], s[2], s[3], s[4])
    msk_batch = msk_batch.reshape(s[0] * s[1], s[2], s[3], s[4])
    if orient == "left":                                            # 1158-1162
        target_x = target_x - targetoff_x / 6.0
    elif orient == "right":
        target_x = target_x + targetoff_x / 6.0
    tx = (-target_x + 0.5) * 2                                      # 1164-1165
    ty = (-target_y + 0.5) * 2
    sin, cos = torch.sin(angle), torch.cos(angle)
    theta = torch.zeros(anglesize, 2, 3)                            # 1171-1178
    theta[:, 0, 0] = cos / scale
    theta[:, 0, 1] = sin / scale
    theta[:, 0, 2] = tx * cos / scale + ty * sin / scale
    theta[:, 1, 0] = -sin / scale
    theta[:, 1, 1] = cos / scale
    theta[:, 1, 2] = -tx * sin / scale + ty * cos / scale
    grid = F.affine_grid(theta, adv_batch.shape, align_corners=False)     # 1180
    adv_t = F.grid_sample(adv_batch, grid, align_corners=False)           # 1183-1184
    msk_t = F.grid_sample(msk_batch, grid, align_corners=False)
    adv_t = adv_t.view(s[0], s[1], s[2], s[3], s[4])
    msk_t = msk_t.view(s[0], s[1], s[2], s[3], s[4])
    adv_t = torch.clamp(adv_t, 0.0, 1.)                             # 1227
    return adv_t * msk_t                                            # 1230
