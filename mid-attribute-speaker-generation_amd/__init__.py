"""MI355X-native FastSpeech2 + TacoSpawn-GMM training step.

Drop-in for the reference's ``model.fastspeech2.FastSpeech2`` / ``model.loss`` /
``model.optimizer.ScheduledOptim`` hot path.  Compute runs in hand-written
gfx950 HIP kernels behind the C-ABI library ``csrc/libfs2hip.so`` (declared in
``include/fs2hip.h``); PyTorch only provides device memory, streams, autograd plumbing and
``torch.distributed``.
"""
from . import config, data, seeded  # noqa: F401  (CPU-safe modules)
