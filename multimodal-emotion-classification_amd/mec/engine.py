"""Batched tensor API over the C ABI: device-resident inputs in, device tensors out.

Torch owns device memory and the stream (plumbing); all arithmetic runs in the HIP
kernels of libmec_hip.so. Each call validates shapes/dtypes/devices on the host before
any launch, and raises MecError when the library or a GPU is unavailable — there is no
CPU fallback on this path.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np
import torch

from . import _lib, synthetic
from ._lib import MecError

TAG_BERT_FFN2 = 5  # launch class of BERT's FFN2 GEMM (mec_common.h Tag)
TAG_BERT_QKV = 1  # ... and of its QKV GEMM
TAG_BERT_OPROJ = 3  # ... and of its attention output projection

KINDS = synthetic.KIND_IDS


def _ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check_tensor(name, t, dtype, shape, device):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f'{name}: expected a torch.Tensor, got {type(t).__name__}')
    if t.device != device:
        raise ValueError(f'{name}: on {t.device}, expected {device}')
    if t.dtype != dtype:
        raise TypeError(f'{name}: dtype {t.dtype}, expected {dtype}')
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f'{name}: shape {tuple(t.shape)}, expected {tuple(shape)}')
    if not t.is_contiguous():
        raise ValueError(f'{name}: must be contiguous')


def require_gpu(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise MecError('no ROCm GPU visible: the HIP inference path has no CPU fallback')
    if device is None:
        return torch.device('cuda', torch.cuda.current_device())
    d = torch.device(device)
    if d.type != 'cuda':
        raise MecError(f'device {d}: the HIP inference path runs on a ROCm GPU only')
    return torch.device('cuda', d.index if d.index is not None else torch.cuda.current_device())


class HipModel:
    """Owns one mec_model handle (packed device weights + workspace).

    fp32x3 handles answer on data outside their activation-plane envelope instead of failing: the
    checked paths (`checked`, and through it the drop-in classes and FusedPipeline.check) notice a
    raised range flag (mec_model_check == MEC_ERR_X3_RANGE), re-run the batch on an fp32 handle of the
    same weights (`fp32_twin`, the exact-fp32 HIP engine, created on first use) and re-create this
    handle with 8 more binades of plane headroom (`x3_headroom`), so later batches run fp32x3 again."""

    kind: str = ''
    X3_HEADROOM_STEP = 8  # binades added per range trip (mec_create_opt "x3_headroom", at most 24)

    def __init__(self, weights=None, seed: int = 1234, device=None, precision: str = 'f16', opts=None):
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_lib.PRECISIONS)}, got {precision!r}")
        self.lib = _lib.load()
        self.device = require_gpu(device)
        self.precision = precision
        # the weights dict (synthetic weights are cached per (kind, seed), so this holds no copy): a range
        # trip re-creates the handle from it
        self._w = weights if weights is not None else synthetic.weights(self.kind, seed)
        self._seed = seed
        self._copts = dict(opts or {})  # creation-time knobs (mec_create_opt)
        self._knobs = []                # set_option calls, replayed onto a re-created handle
        self._twin = None
        self.x3_reruns = 0              # batches re-run on the fp32 engine after a range trip
        self._lock = threading.Lock()
        self.handle = None
        self.handle = self._create(self._copts)

    def _create(self, copts):
        blob = synthetic.pack(self.kind, self._w)
        want = self.lib.mec_blob_size(KINDS[self.kind])
        if blob.size != want:
            raise MecError(f'{self.kind}: blob has {blob.size} floats, library expects {want}')
        h = ctypes.c_void_p()
        torch.cuda.set_device(self.device)
        spec = ','.join(f'{k}={int(v)}' for k, v in copts.items()).encode()
        _lib.check(self.lib.mec_create_opt(KINDS[self.kind], blob.ctypes.data_as(_lib.c_fp), blob.size,
                                           self.device.index, _lib.PRECISIONS[self.precision], spec, ctypes.byref(h)),
                   f'mec_create({self.kind}, {self.precision})')
        return h

    def close(self):
        if getattr(self, 'handle', None):
            self.lib.mec_destroy(self.handle)
            self.handle = None
        if getattr(self, '_twin', None) is not None:
            self._twin.close()
            self._twin = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, key: str, value: int):
        """One tuning knob of THIS handle (mec_model_set_option; include/mec.h lists them)."""
        _lib.check(self.lib.mec_model_set_option(self.handle, key.encode(), int(value)), f'set_option({key}={value})')
        self._knobs.append((key, int(value)))

    def check(self):
        """Raise MecError if a kernel of this handle flagged an error after the fact since the
        last check (mec_model_check; speech: an expired hand-off wait, whose forward's probs are
        NaN; fp32x3: X3RangeError, an activation outside the planes' range). Call once the stream
        that ran the forwards has been synchronized."""
        _lib.check(self.lib.mec_model_check(self.handle), f'{self.kind} forward')

    def x3_report(self) -> str:
        """The activation-plane exponents this fp32x3 handle was created with (mec_model_x3_report)."""
        r = self.lib.mec_model_x3_report(self.handle)
        return r.decode() if r else ''

    @property
    def x3_headroom(self) -> int:
        return int(self._copts.get('x3_headroom', 0))

    def fp32_twin(self):
        """An exact-fp32 handle of the same kind and weights (created on first use)."""
        if self._twin is None:
            self._twin = type(self)(self._w, self._seed, self.device, 'fp32')
        return self._twin

    def x3_widen(self):
        """Re-create this fp32x3 handle with X3_HEADROOM_STEP more binades of plane headroom."""
        hr = min(24, self.x3_headroom + self.X3_HEADROOM_STEP)
        if hr == self.x3_headroom:
            return
        copts = dict(self._copts, x3_headroom=hr)
        with self._lock:
            torch.cuda.synchronize(self.device)  # nothing of the old handle may still run
            h = self._create(copts)
            old, self.handle, self._copts = self.handle, h, copts
            self.lib.mec_destroy(old)
            for k, v in self._knobs:
                _lib.check(self.lib.mec_model_set_option(self.handle, k.encode(), v), f'set_option({k}={v})')

    def recover(self, method: str, args, outs):
        """After a synchronized forward `getattr(self, method)(*args)` -> `outs`: check the handle; on an
        fp32x3 range trip re-run the call on the fp32 twin, copy its results into `outs` (in place), widen
        this handle, and return True. Other errors raise as `check` does."""
        rc = self.lib.mec_model_check(self.handle)
        if rc == 0:
            return False
        if rc != _lib.ERR_X3_RANGE or self.precision != 'fp32x3':
            _lib.check(rc, f'{self.kind} forward')
        twin = self.fp32_twin()
        with torch.cuda.device(self.device):
            res = getattr(twin, method)(*args)
            for o, r in zip(outs, res):
                o.copy_(r)
            torch.cuda.synchronize(self.device)
        twin.check()
        self.x3_reruns += 1
        self.x3_widen()
        return True

    def checked(self, method: str, *args):
        """`getattr(self, method)(*args)`, synchronized and checked: an fp32x3 range trip is answered by
        the fp32 engine (recover) instead of raising. Returns the forward's outputs."""
        outs = getattr(self, method)(*args)
        torch.cuda.synchronize(self.device)
        self.recover(method, args, outs)
        return outs

    def gemm_tile(self, M: int, N: int, K: int, amode: int = 0) -> int:
        """The tile this handle's autotuner chose for a GEMM shape it has run (0 = not seen)."""
        return self.lib.mec_model_gemm_query(self.handle, amode, M, N, K)

    # hipEvent timing hook
    def prof_enable(self, tag: str | int):
        t = _lib.TAGS[tag] if isinstance(tag, str) else int(tag)
        _lib.check(self.lib.mec_prof_enable(self.handle, t), 'mec_prof_enable')

    def prof_read(self):
        ms = ctypes.c_double()
        n = ctypes.c_int()
        _lib.check(self.lib.mec_prof_read(self.handle, ctypes.byref(ms), ctypes.byref(n)), 'mec_prof_read')
        return ms.value, n.value

    def _empty(self, *shape, dtype=torch.float32):
        return torch.empty(shape, dtype=dtype, device=self.device)


class SpeechEncoder(HipModel):
    kind = 'speech'

    def forward(self, x: torch.Tensor):
        """x f32 [B,56] raw features -> (feat [B,64], logits [B,7], probs [B,7])."""
        B = x.shape[0] if x.dim() == 2 else -1
        _check_tensor('x', x, torch.float32, (B, 56), self.device)
        feat, logits, probs = self._empty(B, 64), self._empty(B, 7), self._empty(B, 7)
        with self._lock:
            _lib.check(self.lib.mec_speech_fwd(self.handle, _ptr(x), B, _ptr(feat), _ptr(logits), _ptr(probs),
                                               _stream(self.device)), 'mec_speech_fwd')
        return feat, logits, probs


class TextEncoder(HipModel):
    kind = 'text'

    VOCAB = 30522  # bert-base-uncased word embeddings

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        # BERT's GEMMs walk their tiles in groups of 4 M panels per XCD (the handle default is 8, which
        # ResNet50 keeps): fp32x3 fused step 25.51 -> 25.35 and 25.38 -> 25.31 ms, BERT alone 17.44 ->
        # 17.32 ms, f16 fused step 10.76 -> 10.74 ms; the same bits (profiles/r05y_ab_groupm_*.txt,
        # profiles/r05z_ab_groupm_*.txt)
        self.set_option('gemm_glds_group_m', 4)

    def forward(self, ids: torch.Tensor, mask: torch.Tensor, check_ids: bool = False):
        """ids/mask int32 [B,128] -> (cls [B,768], logits [B,7], probs [B,7]).

        check_ids: raise ValueError for ids outside [0, 30522) like nn.Embedding does (one
        device min/max reduction and a host sync; the batched hot path skips it, and the kernel
        then clamps out-of-range ids)."""
        if ids.dim() != 2:
            raise ValueError('ids: expected [B, L]')
        B, L = ids.shape
        if L != 128:
            raise ValueError('ids: L must be 128 (padding=max_length, Config.MAX_TEXT_LENGTH)')
        _check_tensor('ids', ids, torch.int32, (B, L), self.device)
        _check_tensor('mask', mask, torch.int32, (B, L), self.device)
        if check_ids and B:
            lo, hi = (int(v) for v in torch.aminmax(ids))
            if lo < 0 or hi >= self.VOCAB:
                raise ValueError(f'ids: token id out of range [0, {self.VOCAB}): min {lo}, max {hi}')
        cls, logits, probs = self._empty(B, 768), self._empty(B, 7), self._empty(B, 7)
        with self._lock:
            _lib.check(self.lib.mec_text_fwd(self.handle, _ptr(ids), _ptr(mask), B, L, _ptr(cls), _ptr(logits),
                                             _ptr(probs), _stream(self.device)), 'mec_text_fwd')
        return cls, logits, probs


class ImageEncoder(HipModel):
    kind = 'image'

    def forward(self, gray: torch.Tensor):
        """gray u8 [B,48,48] -> (feat [B,512], logits [B,7], probs [B,7])."""
        B = gray.shape[0] if gray.dim() == 3 else -1
        _check_tensor('gray', gray, torch.uint8, (B, 48, 48), self.device)
        feat, logits, probs = self._empty(B, 512), self._empty(B, 7), self._empty(B, 7)
        with self._lock:
            _lib.check(self.lib.mec_image_fwd(self.handle, _ptr(gray), B, _ptr(feat), _ptr(logits), _ptr(probs),
                                              _stream(self.device)), 'mec_image_fwd')
        return feat, logits, probs

    def forward_u8(self, img: torch.Tensor):
        """img u8 [B,H,W,C] with (H,W,C) in {(48,48,1), (224,224,1), (224,224,3)}."""
        if img.dim() == 3:
            img = img.unsqueeze(-1)
        if img.dim() != 4 or tuple(img.shape[1:]) not in ((48, 48, 1), (224, 224, 1), (224, 224, 3)):
            raise ValueError(f'img: shape {tuple(img.shape)} not in [B,48,48,1] / [B,224,224,1] / [B,224,224,3]')
        B, H, W, C = img.shape
        _check_tensor('img', img, torch.uint8, (B, H, W, C), self.device)
        feat, logits, probs = self._empty(B, 512), self._empty(B, 7), self._empty(B, 7)
        with self._lock:
            _lib.check(self.lib.mec_image_fwd_u8(self.handle, _ptr(img), B, H, W, C, _ptr(feat), _ptr(logits),
                                                 _ptr(probs), _stream(self.device)), 'mec_image_fwd_u8')
        return feat, logits, probs


class MobileNetImageEncoder(ImageEncoder):
    """The same image entry points on the MobileNetV2 backbone (csrc/mobilenet.hip)."""
    kind = 'image_mbv2'


IMAGE_BACKBONES = {'resnet50': ImageEncoder, 'mobilenet_v2': MobileNetImageEncoder}

AUDIO_KIND = 5  # include/mec.h MEC_AUDIO
N_FFT, HOP, N_MELS = 2048, 512, 128  # librosa defaults the reference never overrides


class AudioFeaturizer(HipModel):
    """preprocess_audio's 56-d speech features (preprocessing/audio_preprocessing.py:22-46:
    mean MFCC-40 | mean chroma-12 | mean zcr, centroid, rolloff, rms) computed on the GPU
    (csrc/audio.hip) for a batch of fixed-length waveforms (load_audio's pad/trim applied)."""
    kind = 'audio'

    def __init__(self, sample_rate: int = 22050, n_mfcc: int = 40, device=None):
        self.lib = _lib.load()
        self.device = require_gpu(device)
        self.precision = 'fp32'
        self.sample_rate, self.n_mfcc = int(sample_rate), int(n_mfcc)
        self._knobs, self._twin, self._copts, self.x3_reruns = [], None, {}, 0
        self.n_features = self.n_mfcc + 16
        blob = np.array([sample_rate, N_FFT, HOP, N_MELS, n_mfcc], np.float32)
        h = ctypes.c_void_p()
        torch.cuda.set_device(self.device)
        _lib.check(self.lib.mec_create_ex(AUDIO_KIND, blob.ctypes.data_as(_lib.c_fp), blob.size, self.device.index,
                                          _lib.PRECISIONS['fp32'], ctypes.byref(h)), 'mec_create(audio)')
        self.handle = h
        self._lock = threading.Lock()

    def forward(self, wave: torch.Tensor, return_tuning: bool = False):
        """wave f32 [B, n] -> features f32 [B, n_mfcc + 16] (and the chroma tuning [B])."""
        if wave.dim() != 2:
            raise ValueError('wave: expected [B, n_samples]')
        B, n = wave.shape
        _check_tensor('wave', wave, torch.float32, (B, n), self.device)
        feat = self._empty(B, self.n_features)
        tun = self._empty(B) if return_tuning else None
        with self._lock:
            _lib.check(self.lib.mec_audio_fwd(self.handle, _ptr(wave), B, n, _ptr(feat), _ptr(tun),
                                              _stream(self.device)), 'mec_audio_fwd')
        return (feat, tun) if return_tuning else feat


class FusionHead(HipModel):
    kind = 'fusion'

    def forward(self, s_feat, t_feat, i_feat, s_pred, t_pred, i_pred):
        """-> (logits [B,7], probs [B,7], attn_w [B,3], dec_w [B,3])."""
        B = s_feat.shape[0]
        for n, t, d in (('s_feat', s_feat, 64), ('t_feat', t_feat, 768), ('i_feat', i_feat, 512),
                        ('s_pred', s_pred, 7), ('t_pred', t_pred, 7), ('i_pred', i_pred, 7)):
            _check_tensor(n, t, torch.float32, (B, d), self.device)
        logits, probs, aw, dw = self._empty(B, 7), self._empty(B, 7), self._empty(B, 3), self._empty(B, 3)
        with self._lock:
            _lib.check(self.lib.mec_fusion_fwd(self.handle, _ptr(s_feat), _ptr(t_feat), _ptr(i_feat), _ptr(s_pred),
                                               _ptr(t_pred), _ptr(i_pred), B, _ptr(logits), _ptr(probs), _ptr(aw),
                                               _ptr(dw), _stream(self.device)), 'mec_fusion_fwd')
        return logits, probs, aw, dw


def fuse_weighted(s=None, t=None, i=None, device=None) -> torch.Tensor:
    """Weighted-average fallback on the GPU (float64) -> [B,7] f64; None = missing modality."""
    present = [x for x in (s, t, i) if x is not None]
    lib = _lib.load()
    dev = present[0].device if present else require_gpu(device)
    B = present[0].shape[0] if present else 1
    for n, x in (('s', s), ('t', t), ('i', i)):
        if x is not None:
            _check_tensor(n, x, torch.float32, (B, 7), dev)
    out = torch.empty((B, 7), dtype=torch.float64, device=dev)
    _lib.check(lib.mec_fuse_weighted(_ptr(s), _ptr(t), _ptr(i), B, _ptr(out), _stream(dev)), 'mec_fuse_weighted')
    return out


def fuse_weighted_f64(s=None, t=None, i=None, device=None) -> torch.Tensor:
    """Same as fuse_weighted with float64 [B,7] inputs (per-request Python floats)."""
    present = [x for x in (s, t, i) if x is not None]
    lib = _lib.load()
    dev = present[0].device if present else require_gpu(device)
    B = present[0].shape[0] if present else 1
    for n, x in (('s', s), ('t', t), ('i', i)):
        if x is not None:
            _check_tensor(n, x, torch.float64, (B, 7), dev)
    out = torch.empty((B, 7), dtype=torch.float64, device=dev)
    _lib.check(lib.mec_fuse_weighted_f64(_ptr(s), _ptr(t), _ptr(i), B, _ptr(out), _stream(dev)),
               'mec_fuse_weighted_f64')
    return out


# Packed per-sample result row gathered across ranks: 3x7 modality probs,
# 7 fused probs, 3 attention weights, 3 decision weights = 34 floats.
ROW = 34


class FusedPipeline:
    """The whole tri-modal path: speech + text + image encoders, then the fusion model.

    BERT runs on a high-priority stream (text_priority; else the caller's stream); speech and
    the image backbone run concurrently on a second HIP stream at normal priority, so BERT's
    workgroups are dispatched first and the image kernels fill the CUs that BERT's GEMM tails
    and its LayerNorm/attention kernels leave idle (+1.5% over equal priorities). The first
    call runs everything serially so each GEMM shape is autotuned in isolation.

    pipelined=True (the default with concurrent=True): the fusion model (and the caller's
    `epilogue`, e.g. packing and the all-gather) runs on a third stream that waits for both
    encoder streams, and the caller's stream does NOT wait for it. Consecutive batches
    therefore overlap: batch i's fusion (a latency-bound kernel of ~128 workgroups) runs
    under batch i+1's BERT instead of idling the GPU between them. Every batch's work is still
    done; outputs are ready once `wait()` (or a device synchronize) returns.
    """

    def __init__(self, seed: int = 1234, device=None, weights=None, concurrent: bool = True,
                 image_backbone: str = 'resnet50', pipelined: bool = True, text_priority: bool = True,
                 image_priority: bool = False, precision: str = 'f16'):
        weights = weights or {}
        self.precision = precision
        self.speech = SpeechEncoder(weights.get('speech'), seed, device)
        self.text = TextEncoder(weights.get('text'), seed, device, precision)
        self.image = IMAGE_BACKBONES[image_backbone](weights.get('image'), seed, device, precision)
        self.fusion = FusionHead(weights.get('fusion'), seed, device)
        self.device = self.speech.device
        self.concurrent = concurrent
        self.pipelined = concurrent and pipelined
        # image_priority (A/B): the speech + image stream at high priority instead, BERT on its
        # own normal-priority stream
        self._side = (torch.cuda.Stream(device=self.device, priority=-1 if image_priority else 0)
                      if concurrent else None)
        self._tail = torch.cuda.Stream(device=self.device) if self.pipelined else None
        # text_priority: BERT on its own high-priority stream, so its workgroups are dispatched
        # ahead of the image stream's and the image kernels fill the CUs BERT leaves idle
        self._text = (torch.cuda.Stream(device=self.device, priority=0 if image_priority else -1)
                      if (concurrent and (text_priority or image_priority)) else None)
        self._tuned = set()  # batch sizes whose GEMM shapes were autotuned (serially)
        self._last, self._since_check = None, 0
        if concurrent and precision == 'f16':
            # BERT FFN2 (M = 128 B, N = 768, K = 3072) on the 256 x 256 ping-pong tile beside the
            # image stream: BERT alone runs it fastest on 128 x 128 (the autotuner's pick, text
            # 7.90 vs 8.02 ms at B = 256), but in the concurrent step the 4x fewer, larger tiles
            # win: 11.10 vs 11.37 ms per step (interleaved A/B, tools/gpu_ab_tiles.sh,
            # profiles/r02_ab_tiles_fused.txt). Same k order on both tiles: same bits.
            self.text.set_option('gemm_bn_tag', TAG_BERT_FFN2 * 100000 + 40256)
        if concurrent and precision == 'fp32x3':
            # the same for the fp32x3 path: FFN2 on the 256 x 256 K-interleaved split tile (384 tiles,
            # 1.5 rounds of 256 CUs: the image stream fills the half-empty round) instead of the
            # autotuner's 128 x 128 / 256 x 128 pick: 26.62 vs 27.49 ms per step (interleaved A/B,
            # tools/gpu_ab_x3tags.sh, profiles/r03_ab_x3tag_ffn2.txt). Every interleaved tile gives
            # the same bits.
            self.text.set_option('gemm_x3_tag', TAG_BERT_FFN2 * 100000 + 70256)
            # the O-projection (N = 768) the same way, since the fused QKV kernels share CUs two at a
            # time: 25.00 vs 25.21 ms per step (11 interleaved rounds, profiles/r04_ab_x3tag_oproj2.txt;
            # within 0.3 % in round 3, before that change)
            self.text.set_option('gemm_x3_tag', TAG_BERT_OPROJ * 100000 + 70256)
            # QKV (N = 2304: 1152 tiles, 4.5 rounds) on the same tile, which the autotuner picks alone
            # too but not on every run: 25.45 vs 25.58 ms per step autotuned, 256 x 128 / 128 x 128
            # 25.95 / 25.86 (profiles/r03_ab_x3tag_qkv.txt)
            self.text.set_option('gemm_x3_tag', TAG_BERT_QKV * 100000 + 70256)

    def forward(self, x_speech, ids, mask, gray, epilogue=None):
        """One batch through the path -> dict of per-modality and fusion outputs (and, with
        `epilogue`, ``(outputs, epilogue(outputs))``, the callable run on the fusion's stream)."""
        main = torch.cuda.current_stream(self.device)
        B = int(ids.shape[0])
        if not self.concurrent or B not in self._tuned:
            # a batch size not seen yet runs serially on one stream, so each new GEMM shape is
            # autotuned alone (not against the other encoder's kernels)
            for st in (self._side, self._text, self._tail):  # nothing else in flight while tuning
                if st is not None:
                    main.wait_stream(st)
            sf, sl, sp = self.speech.forward(x_speech)
            tf, tl, tp = self.text.forward(ids, mask)
            imf, il, ip = self.image.forward(gray)
            self._tuned.add(B)
            fstream = main
        else:
            side = self._side
            side.wait_stream(main)  # inputs were produced on the main stream
            with torch.cuda.stream(side):
                sf, sl, sp = self.speech.forward(x_speech)
                imf, il, ip = self.image.forward(gray)
            if self._text is not None:
                tstream = self._text
                tstream.wait_stream(main)
                with torch.cuda.stream(tstream):
                    tf, tl, tp = self.text.forward(ids, mask)
                for t in (ids, mask):
                    t.record_stream(tstream)
                if not self.pipelined:
                    main.wait_stream(tstream)
                    for t in (tf, tl, tp):
                        t.record_stream(main)
            else:
                tstream = main
                tf, tl, tp = self.text.forward(ids, mask)
            for t in (x_speech, gray):
                t.record_stream(side)
            if self.pipelined:
                fstream = self._tail
                fstream.wait_stream(tstream)
                fstream.wait_stream(side)
                for t in (sf, sl, sp, imf, il, ip, tf, tl, tp):
                    t.record_stream(fstream)
            else:
                main.wait_stream(side)
                for t in (sf, sl, sp, imf, il, ip):
                    t.record_stream(main)
                fstream = main
        with torch.cuda.stream(fstream):
            fl, fp, aw, dw = self.fusion.forward(sf, tf, imf, sp, tp, ip)
            out = {'speech': (sf, sl, sp), 'text': (tf, tl, tp), 'image': (imf, il, ip),
                   'fusion': (fl, fp, aw, dw)}
            extra = epilogue(out) if epilogue is not None else None
        self._last = {'text': (ids, mask), 'image': (gray,), 'out': out}  # check() repairs this batch
        self._since_check += 1
        return out if epilogue is None else (out, extra)

    def wait(self, stream=None):
        """Make `stream` (default: the current one) wait for the last batch's fusion."""
        if self.pipelined:
            (stream or torch.cuda.current_stream(self.device)).wait_stream(self._tail)

    def check(self):
        """Synchronize the device, then check every handle (mec_model_check): raise MecError for an
        after-the-fact kernel error. An fp32x3 range trip of the text or image handle is answered instead
        of raised when one batch ran since the last check: that encoder is re-run on its fp32 twin, its
        outputs and the fusion's are overwritten in place in the dict `forward` returned (an `epilogue`'s
        results, computed before, are not), and the handle is re-created with more plane headroom
        (HipModel.recover). With several batches since the last check a trip raises X3RangeError (it
        cannot say which batch). Returns the modalities that were re-run."""
        torch.cuda.synchronize(self.device)
        last, n, redo = self._last, self._since_check, []
        self._since_check = 0
        for name, m in (('text', self.text), ('image', self.image)):
            if last is not None and n == 1 and m.precision == 'fp32x3':
                if m.recover('forward', last[name], last['out'][name]):
                    redo.append(name)
            else:
                m.check()
        self.speech.check()
        self.fusion.check()
        if redo:
            o = last['out']
            (sf, _, sp), (tf, _, tp), (imf, _, ip) = o['speech'], o['text'], o['image']
            for d, r in zip(o['fusion'], self.fusion.forward(sf, tf, imf, sp, tp, ip)):
                d.copy_(r)
            torch.cuda.synchronize(self.device)
        return redo

    @staticmethod
    def pack_rows(out) -> torch.Tensor:
        sp, tp, ip = out['speech'][2], out['text'][2], out['image'][2]
        _, fp, aw, dw = out['fusion']
        return torch.cat([sp, tp, ip, fp, aw, dw], dim=1)

    def models(self):
        return [self.speech, self.text, self.image, self.fusion]

    def set_option(self, key: str, value: int):
        """Set a tuning knob on every handle of the pipeline that knows it."""
        for m in self.models():
            m.set_option(key, value)


def to_device(a: np.ndarray, device) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:
        a = a.copy()
    return torch.from_numpy(a).to(device)
