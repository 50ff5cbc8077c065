"""ORACLE (test infrastructure only): image path = PIL transform + ResNet50 + head, fp32.

Restates inference/image_inference.py:
  transform  Resize((224,224)) -> ToTensor -> Normalize(ImageNet)          :28-32, :112-113
             (resize is PIL-exact: oracle/resize.py)
  network    torchvision resnet50(weights=None) (:57): conv7x7/2 + BN(1e-5) + ReLU +
             maxpool3x3/2, Bottleneck v1.5 x [3,4,6,3] (stride on the 3x3 conv,
             downsample = 1x1 conv/s + BN on block 0), avgpool
  head       fc = Dropout, Linear(2048,512), ReLU, Dropout, Linear(512,7)   :59-65
  feature    fc[2] ReLU output, 512-d (ImageEmotionModel.extract_features :70-90)
  probs      softmax(logits) (:118, :143); label = Config.EMOTIONS[argmax] (:121-123)
torchvision is absent: the network is parity-unpinned beyond this restatement.
"""
import numpy as np
import torch
import torch.nn.functional as F

from .resize import resize_bilinear_u8, to_normalized_tensor

LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]


@torch.no_grad()
def backbone(w, x: torch.Tensor) -> torch.Tensor:
    g = lambda n: torch.from_numpy(np.asarray(w[n], np.float32))

    def bn(t, p):
        return F.batch_norm(t, g(p + '.running_mean'), g(p + '.running_var'), g(p + '.weight'),
                            g(p + '.bias'), training=False, eps=1e-5)

    x = F.relu(bn(F.conv2d(x, g('base.conv1.weight'), stride=2, padding=3), 'base.bn1'))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, (wd, nb, st) in enumerate(LAYERS):
        for b in range(nb):
            p = f'base.layer{li + 1}.{b}.'
            s = st if b == 0 else 1
            y = F.relu(bn(F.conv2d(x, g(p + 'conv1.weight')), p + 'bn1'))
            y = F.relu(bn(F.conv2d(y, g(p + 'conv2.weight'), stride=s, padding=1), p + 'bn2'))
            y = bn(F.conv2d(y, g(p + 'conv3.weight')), p + 'bn3')
            idn = bn(F.conv2d(x, g(p + 'downsample.0.weight'), stride=s), p + 'downsample.1') if b == 0 else x
            x = F.relu(y + idn)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def normalized_from_resized(resized_u8: np.ndarray) -> np.ndarray:
    """u8 [B,224,224] (gray) or [B,224,224,3] (RGB), already PIL-resized -> ToTensor +
    Normalize float32 [B,3,224,224] (image_inference.py:30-31)."""
    a = np.asarray(resized_u8, np.uint8)
    if a.ndim == 3:
        return to_normalized_tensor(a)
    mean = np.array([0.485, 0.456, 0.406], np.float32)
    std = np.array([0.229, 0.224, 0.225], np.float32)
    x = a.astype(np.float32).transpose(0, 3, 1, 2) / np.float32(255.0)
    return ((x - mean[None, :, None, None]) / std[None, :, None, None]).astype(np.float32)


@torch.no_grad()
def head(w, pooled: torch.Tensor):
    g = lambda n: torch.from_numpy(np.asarray(w[n], np.float32))
    feat = F.relu(F.linear(pooled, g('base.fc.1.weight'), g('base.fc.1.bias')))
    logits = F.linear(feat, g('base.fc.4.weight'), g('base.fc.4.bias'))
    return feat.numpy().copy(), logits.numpy().copy(), torch.softmax(logits, dim=-1).numpy().copy()


@torch.no_grad()
def forward_resized(w, resized_u8: np.ndarray):
    """Already-resized u8 image(s) -> (feat512, logits, probs)."""
    return head(w, backbone(w, torch.from_numpy(normalized_from_resized(resized_u8))))


@torch.no_grad()
def forward(w, gray_u8: np.ndarray, return_resized: bool = False):
    """gray u8 [B,48,48] -> (feat512 [B,512], logits [B,7], probs [B,7]) float32 numpy."""
    resized = resize_bilinear_u8(gray_u8)
    x = torch.from_numpy(to_normalized_tensor(resized))
    out = head(w, backbone(w, x))
    return out + (resized,) if return_resized else out
