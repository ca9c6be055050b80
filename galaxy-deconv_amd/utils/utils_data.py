"""Drop-in for reference ``utils/utils_data.py``: the dataset API (``Galaxy_Dataset`` :44-103,
``get_dataloader`` :106-136) plus its two helpers, with the packed-batch ingest path of
``gdeconv.ingest`` beside it (``pack_dataset``, ``PackedGalaxies``, ``DeviceBatches``)."""
import torch
import torch.nn.functional as F

from gdeconv.ingest import (DeviceBatches, Galaxy_Dataset, PackedGalaxies, get_dataloader,  # noqa: F401
                            pack_dataset, write_pack)


def get_flux(ab_magnitude, exp_time, zero_point, gain, qe):
    """Flux in ADU from an AB magnitude (:10-24): t * zp * 10^(-0.4 (m - 24)) * qe / gain."""
    return exp_time * zero_point * 10 ** (-0.4 * (ab_magnitude - 24)) * qe / gain


def down_sample(input, rate=4):
    """[H, W] -> [H/rate, W/rate] by a rate x rate box average (:27-41; a stride-`rate` conv)."""
    w = torch.full((1, 1, rate, rate), 1.0 / (rate ** 2), dtype=input.dtype, device=input.device)
    return F.conv2d(input[None, None], w, stride=rate)[0, 0]


def __getattr__(name):  # names this drop-in does not define come from the reference module
    from gdeconv import refpath
    return refpath.attr(__name__, name)
