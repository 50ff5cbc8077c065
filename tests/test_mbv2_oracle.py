"""CPU: the MobileNetV2 oracle (oracle/image_mbv2.py) and its weight spec.

torchvision is absent and the reference has no MobileNetV2 code (README.md:13 only), so the
restatement is checked two ways that need neither: (1) the spec's parameter count equals
torchvision mobilenet_v2's (3,504,872 with its 1000-class classifier, i.e. 2,223,872 in
`features`) plus the reference-style 1280->512->7 head; (2) a module built with torchvision's
nesting (features[i].conv[j], Conv2dNormActivation = Sequential(conv, bn, ReLU6)) accepts
the spec's state_dict with strict=True and computes what the functional oracle computes.
"""
import numpy as np
import torch
from torch import nn

from mec import synthetic as syn
from oracle import image_mbv2 as o_mb


def _cna(cin, cout, k, s=1, groups=1):
    return nn.Sequential(nn.Conv2d(cin, cout, k, s, (k - 1) // 2, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU6())


class _IR(nn.Module):
    def __init__(self, t, cin, hid, cout, s):
        super().__init__()
        layers = [] if t == 1 else [_cna(cin, hid, 1)]
        layers += [_cna(hid, hid, 3, s, groups=hid), nn.Conv2d(hid, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        self.conv = nn.Sequential(*layers)
        self.res = s == 1 and cin == cout

    def forward(self, x):
        return x + self.conv(x) if self.res else self.conv(x)


class _Base(nn.Module):
    def __init__(self):
        super().__init__()
        feats = [_cna(3, 32, 3, 2)] + [_IR(*b) for b in syn.mbv2_blocks()] + [_cna(320, 1280, 1)]
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Sequential(nn.Dropout(0.5), nn.Linear(1280, 512), nn.ReLU(), nn.Dropout(0.3),
                                        nn.Linear(512, 7))

    def forward(self, x):
        x = nn.functional.adaptive_avg_pool2d(self.features(x), 1).flatten(1)
        return self.classifier(x)


class _Model(nn.Module):
    def __init__(self):
        super().__init__()
        self.base = _Base()


def test_spec_parameter_count():
    spec = syn.image_mbv2_spec()
    n = sum(int(np.prod(sh)) for name, sh, _, _ in spec if 'running' not in name)
    head = 1280 * 512 + 512 + 512 * 7 + 7
    assert n - head == 3504872 - (1280 * 1000 + 1000)  # torchvision mobilenet_v2 features
    assert [b[1:] for b in syn.mbv2_blocks()][:3] == [(32, 32, 16, 1), (16, 96, 24, 2), (24, 144, 24, 1)]
    assert len(syn.mbv2_blocks()) == 17


def test_oracle_matches_torchvision_structured_module():
    w = syn.weights('image_mbv2')
    m = _Model().eval()
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in w.items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected
    assert all(k.endswith('num_batches_tracked') for k in missing)
    gray = syn.image_inputs(2, seed=3)
    from oracle.resize import resize_bilinear_u8, to_normalized_tensor
    x = torch.from_numpy(to_normalized_tensor(resize_bilinear_u8(gray)))
    with torch.no_grad():
        ref = m.base(x).numpy()
    _, logits, probs = o_mb.forward(w, gray)
    assert np.abs(logits - ref).max() < 1e-4


def test_golden_fixture_is_current(golden):
    g = golden('image_mbv2.npz')
    f, l, p = o_mb.forward(syn.weights('image_mbv2', int(g['wseed'])), g['gray'])
    assert np.abs(l - g['logits']).max() < 1e-5
    assert np.array_equal(p.argmax(1), g['probs'].argmax(1))


def test_blob_size_matches_library():
    from mec import _lib
    lib = _lib.load()
    assert lib.mec_blob_size(syn.KIND_IDS['image_mbv2']) == syn.blob_size('image_mbv2')
