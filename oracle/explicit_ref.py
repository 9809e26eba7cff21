"""CPU restatement of the explicit render path's pre-raster steps (TEST INFRASTRUCTURE ONLY).

  * gs_mask  <- scene/lod_model.py:292-296 set_gs_mask with scene/basic_model.py:192-210
                map_to_int_level ('floor'): level <= clamp(floor(log2(sd / (|x - c| * s)) /
                log2(fork) + extra_level), 0, street_levels - 1)
  * gather   <- scene/basic_model.py:373-383 generate_explicit_gaussians (boolean-mask indexing)

Only tests/ import this module; the product (horizongs_amd.explicit) never does.
"""
from __future__ import annotations

import math

import torch


def gs_mask(xyz, level, extra_level, cam_center, res_scale, standard_dist, fork, street_levels):
    dist = torch.sqrt(torch.sum((xyz - cam_center) ** 2, dim=1)) * res_scale
    pred = torch.log2(standard_dist / dist) / math.log2(fork) + extra_level
    int_level = torch.clamp(torch.floor(pred).int(), 0, street_levels - 1)
    return level.reshape(-1) <= int_level


def gather(mask, xyz, features_dc, features_rest, opacity, scaling, rotation):
    color = torch.cat((features_dc, features_rest), dim=1)[mask]
    return xyz[mask], color, opacity[mask], scaling[mask], rotation[mask]
