"""
Image inference (ResNet50 + 2048->512->7 head) on the MI355X HIP path — drop-in for the
reference's inference/image_inference.py (same class, methods, result dicts, fallback).

The reference transform Resize((224,224)) -> ToTensor -> Normalize (:28-32) and the network
run on the GPU (csrc/resnet.hip): a 48x48 grayscale FER2013 face is resized by a PIL-exact
HIP kernel; any other image is decoded and resized by PIL on the host (the same call
torchvision makes) and uploaded as u8 224x224, gray (1 channel) or RGB (3 channels). The
labels are Config.EMOTIONS[argmax] exactly like the reference (:121-123), including its
class-order quirk against ImageFolder's alphabetical training order.

Added beyond the reference: predict_array(u8 image) and predict_batch(u8 [B,48,48]), and
`backbone='mobilenet_v2'` (README.md:13 names MobileNetV2 as the image model; the reference
code builds ResNet50): the same transform, head, feature and result dicts on a
torchvision-mobilenet_v2 backbone (csrc/mobilenet.hip; parity unpinned, no reference code).
"""

from typing import Dict

import numpy as np

from config import Config
from mec import checkpoints, engine
from mec._lib import MecError


def _to_model_input(image) -> np.ndarray:
    """PIL image -> u8 array [H,W,C] in one of the shapes the HIP path takes."""
    from PIL import Image
    rgb = image.convert('RGB')  # reference :112
    a = np.asarray(rgb, dtype=np.uint8)
    gray = bool((a[..., 0] == a[..., 1]).all() and (a[..., 0] == a[..., 2]).all())
    if gray and a.shape[:2] == (48, 48):
        return np.ascontiguousarray(a[..., :1])  # GPU resize path
    r = np.asarray(rgb.resize((224, 224), Image.BILINEAR), dtype=np.uint8)  # Resize((224,224))
    return np.ascontiguousarray(r[..., :1] if gray else r)


_KINDS = {'resnet50': 'image', 'mobilenet_v2': 'image_mbv2'}


class ImageInference:
    def __init__(self, weights=None, seed=None, device=None, backbone='resnet50', precision=None):
        if backbone not in _KINDS:
            raise ValueError(f'backbone must be one of {sorted(_KINDS)}')
        self.emotions = Config.EMOTIONS
        self.backbone = backbone
        self.model = None
        w = checkpoints.resolve(_KINDS[backbone], weights, seed)
        if w is not None:  # raises MecError without HIP/GPU
            self.model = engine.IMAGE_BACKBONES[backbone](w, device=device,
                                                          precision=checkpoints.precision(precision))
        self.device = self.model.device if self.model is not None else None

    def _fallback(self) -> Dict:
        probs = np.ones(len(self.emotions)) * (0.1 / (len(self.emotions) - 1))
        idx = self.emotions.index('neutral')
        probs[idx] = 0.9
        return {'emotion': 'neutral', 'confidence': float(probs[idx]), 'all_probabilities': probs.tolist()}

    def _forward(self, arr: np.ndarray):
        x = engine.to_device(np.asarray(arr, np.uint8)[None], self.device)
        # synchronized and checked: an fp32x3 batch whose activations leave the planes' range is re-run on
        # the fp32 engine (engine.HipModel.recover), never answered with NaN probs
        feat, logits, probs = self.model.checked('forward_u8', x)
        return feat.cpu().numpy()[0], probs.cpu().numpy()[0]

    @staticmethod
    def _as_dict(emotions, probs: np.ndarray) -> Dict:
        idx = int(np.argmax(probs))
        return {'emotion': emotions[idx], 'confidence': float(probs[idx]), 'all_probabilities': probs.tolist()}

    def predict_array(self, arr) -> Dict:
        """u8 image [48,48] / [48,48,1] / [224,224,1] / [224,224,3] -> result dict."""
        a = np.asarray(arr, np.uint8)
        if a.ndim == 2:
            a = a[..., None]
        return self._as_dict(self.emotions, self._forward(a)[1])

    def predict(self, image_file_path: str) -> Dict:
        if self.model is None:
            return self._fallback()
        try:
            from PIL import Image
            with Image.open(image_file_path) as im:
                arr = _to_model_input(im)
            return self._as_dict(self.emotions, self._forward(arr)[1])
        except MecError:
            raise  # a failing HIP kernel is never hidden behind the fallback
        except Exception as e:
            print(f"Image inference error: {e}")
            return self._fallback()

    def extract_features(self, image_file_path: str):
        """(512-d fc[2] feature, 7 probs) — one forward instead of three."""
        if self.model is None:
            return None, None
        from PIL import Image
        with Image.open(image_file_path) as im:
            arr = _to_model_input(im)
        return self._forward(arr)

    def predict_batch(self, gray):
        """gray: device u8 [B,48,48] -> (feat [B,512], logits [B,7], probs [B,7]). Asynchronous on the
        current stream, except on an fp32x3 handle: there it synchronizes and checks, so a batch outside
        the planes' range is answered by the fp32 engine (engine.HipModel.checked)."""
        if self.model is None:
            raise RuntimeError('image model not loaded')
        if self.model.precision == 'fp32x3':
            return self.model.checked('forward', gray)
        return self.model.forward(gray)
