"""ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of the HiFi-GAN generator forward
(hifigan/models.py:19-178, V1 config) after remove_weight_norm, in plain torch fp32.

Pinned to tests/golden/g9_hifigan.npz (the reference itself on name-seeded weights).
Used by tests as the checker of the HIP vocoder; never imported by the product path."""
import torch
import torch.nn.functional as F

LRELU_SLOPE = 0.1


def generator_forward(sd, h, mel):
    """sd: {key: fp32 tensor} with the reference's post-weight-norm keys; mel (B, 80, T)."""
    x = F.conv1d(mel, sd["conv_pre.weight"], sd["conv_pre.bias"], padding=3)  # models.py:156
    nk = len(h["resblock_kernel_sizes"])
    for i, (u, k) in enumerate(zip(h["upsample_rates"], h["upsample_kernel_sizes"])):
        x = F.leaky_relu(x, LRELU_SLOPE)
        x = F.conv_transpose1d(x, sd[f"ups.{i}.weight"], sd[f"ups.{i}.bias"], stride=u,
                               padding=(k - u) // 2)  # models.py:127-137,159
        xs = None
        for j, (rk, dil) in enumerate(zip(h["resblock_kernel_sizes"],
                                          h["resblock_dilation_sizes"])):
            p = f"resblocks.{i * nk + j}"
            y = x
            for m, d in enumerate(dil):  # ResBlock.forward, models.py:94-100
                xt = F.leaky_relu(y, LRELU_SLOPE)
                xt = F.conv1d(xt, sd[f"{p}.convs1.{m}.weight"], sd[f"{p}.convs1.{m}.bias"],
                              dilation=d, padding=(rk * d - d) // 2)
                xt = F.leaky_relu(xt, LRELU_SLOPE)
                xt = F.conv1d(xt, sd[f"{p}.convs2.{m}.weight"], sd[f"{p}.convs2.{m}.bias"],
                              padding=(rk - 1) // 2)
                y = xt + y
            xs = y if xs is None else xs + y
        x = xs / nk
    x = F.leaky_relu(x)  # default slope 0.01, models.py:167
    x = F.conv1d(x, sd["conv_post.weight"], sd["conv_post.bias"], padding=3)
    return torch.tanh(x)
