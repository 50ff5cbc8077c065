"""ORACLE (test infrastructure only): image path on a MobileNetV2 backbone, fp32.

The reference's README names MobileNetV2 as the image model (README.md:13, :86, :299) but
its code builds ResNet50 (inference/image_inference.py:57); BASELINE config "Image-only:
MobileNetV2 on 48x48x1 FER2013 tensors". This restates that model the way the reference
builds its ResNet50 one, with torchvision's mobilenet_v2(weights=None) as `base`:
  transform  Resize((224,224)) -> ToTensor -> Normalize(ImageNet)   image_inference.py:28-32
             (PIL-exact resize: oracle/resize.py)
  network    torchvision mobilenet_v2 (width 1.0): features[0] = conv3x3/2 3->32 + BN(1e-5)
             + ReLU6; features[1..17] = InvertedResidual(t, c, n, s) x [(1,16,1,1),
             (6,24,2,2), (6,32,3,2), (6,64,4,2), (6,96,3,1), (6,160,3,2), (6,320,1,1)]:
             [1x1 expand + BN + ReLU6 if t != 1] -> 3x3 depthwise/s + BN + ReLU6 -> 1x1
             project + BN (linear bottleneck), + input when stride 1 and cin == cout;
             features[18] = 1x1 320->1280 + BN + ReLU6; global average pool
  head       classifier = Dropout, Linear(1280,512), ReLU, Dropout, Linear(512,7) (the
             reference's fc head, image_inference.py:59-65, on 1280 features)
  feature    classifier[2] ReLU output, 512-d (as ImageEmotionModel.extract_features :70-90)
torchvision is absent and the reference has no MobileNetV2 code: parity unpinned beyond
this restatement (its input transform is PIL-pinned).
"""
import numpy as np
import torch
import torch.nn.functional as F

from .image import normalized_from_resized
from .resize import resize_bilinear_u8, to_normalized_tensor

SETTINGS = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
            (6, 320, 1, 1)]


def blocks():
    out, cin = [], 32
    for t, c, n, s in SETTINGS:
        for i in range(n):
            out.append((t, cin, cin * t, c, s if i == 0 else 1))
            cin = c
    return out


@torch.no_grad()
def backbone(w, x: torch.Tensor) -> torch.Tensor:
    g = lambda n: torch.from_numpy(np.asarray(w[n], np.float32))

    def bn(t, p):
        return F.batch_norm(t, g(p + '.running_mean'), g(p + '.running_var'), g(p + '.weight'),
                            g(p + '.bias'), training=False, eps=1e-5)

    relu6 = lambda t: F.hardtanh(t, 0.0, 6.0)
    x = relu6(bn(F.conv2d(x, g('base.features.0.0.weight'), stride=2, padding=1), 'base.features.0.1'))
    for i, (t, cin, hid, cout, st) in enumerate(blocks()):
        p = f'base.features.{i + 1}.conv.'
        y = x
        if t != 1:
            y = relu6(bn(F.conv2d(y, g(p + '0.0.weight')), p + '0.1'))
            dw, dwbn, pw, pwbn = p + '1.0.weight', p + '1.1', p + '2.weight', p + '3'
        else:
            dw, dwbn, pw, pwbn = p + '0.0.weight', p + '0.1', p + '1.weight', p + '2'
        y = relu6(bn(F.conv2d(y, g(dw), stride=st, padding=1, groups=hid), dwbn))
        y = bn(F.conv2d(y, g(pw)), pwbn)
        x = x + y if (st == 1 and cin == cout) else y
    x = relu6(bn(F.conv2d(x, g('base.features.18.0.weight')), 'base.features.18.1'))
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


@torch.no_grad()
def head(w, pooled: torch.Tensor):
    g = lambda n: torch.from_numpy(np.asarray(w[n], np.float32))
    feat = F.relu(F.linear(pooled, g('base.classifier.1.weight'), g('base.classifier.1.bias')))
    logits = F.linear(feat, g('base.classifier.4.weight'), g('base.classifier.4.bias'))
    return feat.numpy().copy(), logits.numpy().copy(), torch.softmax(logits, dim=-1).numpy().copy()


@torch.no_grad()
def forward_resized(w, resized_u8: np.ndarray):
    """Already-resized u8 image(s) [B,224,224] / [B,224,224,C] -> (feat512, logits, probs)."""
    return head(w, backbone(w, torch.from_numpy(normalized_from_resized(resized_u8))))


@torch.no_grad()
def forward(w, gray_u8: np.ndarray):
    """gray u8 [B,48,48] -> (feat512 [B,512], logits [B,7], probs [B,7]) float32 numpy."""
    x = torch.from_numpy(to_normalized_tensor(resize_bilinear_u8(gray_u8)))
    return head(w, backbone(w, x))
