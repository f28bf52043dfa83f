"""Image losses of the train step (utils/loss_utils.py), restated in torch.

These are the reference's formulations: train.py:244 takes the L1 loss of the batch and, when
`lambda_dssim != 0`, adds `lambda_dssim * (1 - ssim(image, gt))` (train.py:255-257).  The fused L1
kernel the train step uses by default is gs4d_train.kernels.l1_loss; `l1_loss_torch` is its parity
reference and the `fused=False` path.
"""
from math import exp

import torch
import torch.nn.functional as F


def l1_loss_torch(network_output, gt):
    """utils/loss_utils.py:20-21"""
    return torch.abs((network_output - gt)).mean()


def l2_loss(network_output, gt):
    """utils/loss_utils.py:23-24"""
    return ((network_output - gt) ** 2).mean()


def gaussian(window_size, sigma):
    """utils/loss_utils.py:26-28: normalised 1-D Gaussian taps centred on window_size // 2."""
    g = torch.tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)])
    return g / g.sum()


def create_window(window_size, channel):
    """utils/loss_utils.py:30-34: the separable 2-D window (outer product, sigma 1.5), one per channel."""
    w1 = gaussian(window_size, 1.5).unsqueeze(1)
    w2 = w1.mm(w1.t()).float().unsqueeze(0).unsqueeze(0)
    return w2.expand(channel, 1, window_size, window_size).contiguous()


def ssim(img1, img2, window_size=11, size_average=True):
    """utils/loss_utils.py:36-66: SSIM with an 11x11 Gaussian window (sigma 1.5), zero padding, per
    channel (grouped conv), C1 = 0.01^2, C2 = 0.03^2; mean over everything when size_average, else
    the per-image mean."""
    channel = img1.size(-3)
    window = create_window(window_size, channel).to(device=img1.device, dtype=img1.dtype)
    pad = window_size // 2
    mu1 = F.conv2d(img1, window, padding=pad, groups=channel)
    mu2 = F.conv2d(img2, window, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    sigma1_sq = F.conv2d(img1 * img1, window, padding=pad, groups=channel) - mu1_sq
    sigma2_sq = F.conv2d(img2 * img2, window, padding=pad, groups=channel) - mu2_sq
    sigma12 = F.conv2d(img1 * img2, window, padding=pad, groups=channel) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    if size_average:
        return ssim_map.mean()
    return ssim_map.mean(1).mean(1).mean(1)


def psnr(img1, img2):
    """utils/image_utils.py:17-30 without a mask: per-image 20 log10(1 / sqrt(MSE)), shape (B, 1)."""
    mse = ((img1 - img2) ** 2).view(img1.shape[0], -1).mean(1, keepdim=True)
    return 20 * torch.log10(1.0 / torch.sqrt(mse))
