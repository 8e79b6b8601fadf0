"""End-to-end synthesis on the HIP path: FastSpeech2 inference + HiFi-GAN (BASELINE config 5;
SURVEY.md §8 row f1).

``synthesize(model, configs, vocoder, batchs, control_values)`` mirrors ``synthesize.py:104-131``
and the vocoder leg of ``utils/tools.py:synth_samples`` (228-276): for each text batch
``(ids, raw_texts, speakers, texts, src_lens, max_src_len, speaker_meta, accents)`` the model
runs in eval mode with the p/e/d controls, the PostNet mel ``(B, T, 80)`` goes to the vocoder
in its row layout (the reference transposes it to ``(B, 80, T)`` first), and each waveform is
cropped to ``mel_len * hop_length`` samples as int16 PCM.  Figures and .wav files
(``synth_samples``' plotting / ``wavfile.write``) are outside the hot path; the arrays are
returned instead.
"""
import torch

from .dataset import to_device


@torch.no_grad()
def synth_batch(model, vocoder, batch, control_values=(1.0, 1.0, 1.0), hop_length=256,
                max_wav_value=32768.0):
    """One device batch (8-tuple, ``synthesize.py:109-121``) -> (model output tuple,
    list of int16 waveforms cropped to their lengths)."""
    p_c, e_c, d_c = control_values
    speaker_meta = batch[-2].view(batch[-2].shape[0] if batch[-2].dim() > 1 else 1, -1)
    accents = batch[-1]
    head = batch[:-2]
    out = model(*head[2:], p_control=p_c, e_control=e_c, d_control=d_c, accents=accents,
                speaker_meta=speaker_meta)
    post, mel_len = out[1], out[9]
    B, T, C = post.shape
    # length-aware vocoder launches (frames past mel_len + the receptive radius are not
    # computed); the kept samples equal the padded pass of utils/tools.py:264-270
    _, pcm = vocoder.forward_rows(post.reshape(B * T, C), B, T, pcm=True,
                                  max_wav_value=max_wav_value, lengths=mel_len)
    lengths = (mel_len * hop_length).tolist()
    pcm = pcm.view(B, -1)
    wavs = [pcm[i, : lengths[i]].cpu().numpy() for i in range(B)]
    return out, wavs


def synthesize(model, configs, vocoder, batchs, control_values):
    """``synthesize.py:104-131`` over host batches; returns ``[(ids, wavs), ...]``."""
    pp = configs[0]
    hop = pp["stft"]["hop_length"]  # utils/tools.py:267
    audio = pp["audio"]
    dev = next(model.parameters()).device
    model.eval()
    results = []
    for batch in batchs:
        b = to_device(batch, dev)
        _, wavs = synth_batch(model, vocoder, b, control_values, hop, float(audio["max_wav_value"]))
        results.append((batch[0], wavs))
    return results
