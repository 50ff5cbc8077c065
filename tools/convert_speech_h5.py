"""Offline converter: the reference's trained Keras speech model (.h5) -> speech_weights.npz.

The reference trains the speech DNN with TensorFlow 2.13 (requirements.txt:6) and saves it
with `model.save(Config.SPEECH_MODEL_PATH)` (model_training/train_speech_model.py:257), i.e.
the Keras-2 legacy HDF5 layout:

    /model_weights                 attrs: layer_names = [b'dense', b'batch_normalization', ...]
    /model_weights/<layer>         attrs: weight_names = [b'<layer>/kernel:0', ...]
    /model_weights/<layer>/<layer>/kernel:0                              (datasets)

The network (train_speech_model.py:55-90) is 5 x [Dense, BatchNormalization, Activation,
Dropout] + Dense(7). This tool walks `layer_names` in order, keeps the layers that own
weights, and classifies them by their weight names (kernel/bias = Dense, gamma/beta/
moving_mean/moving_variance = BatchNormalization), so Keras' auto-numbered layer names
(dense_3, batch_normalization_7, ...) do not matter. Output names are those of
mec.synthetic.speech_spec(): dense_{i}/kernel, dense_{i}/bias, batch_normalization_{i}/...,
dense_5/..., scaler/mean_, scaler/scale_.

The feature scaler (a joblib pickle of sklearn's StandardScaler, train_speech_model.py:258)
is NOT unpickled here. Export its two arrays once, in the environment that trained it:

    python -c "import joblib, numpy as np; s = joblib.load('models/speech_scaler.pkl'); \
               np.savez('models/speech_scaler.npz', mean_=s.mean_, scale_=s.scale_)"

Needs h5py + numpy (this container: /opt/conda/bin/python3.9):

    /opt/conda/bin/python3.9 tools/convert_speech_h5.py models/speech_model.h5 \
        --scaler models/speech_scaler.npz -o models/speech_weights.npz
"""
import argparse
import sys

import numpy as np

DIMS = [56, 512, 512, 256, 128, 64, 7]
BN_KEYS = ('gamma', 'beta', 'moving_mean', 'moving_variance')


def _s(x):
    return x.decode() if isinstance(x, bytes) else str(x)


def read_layers(path):
    """[(kind, {short_name: array})] for every weighted layer, in model order."""
    import h5py
    out = []
    with h5py.File(path, 'r') as f:
        g = f['model_weights'] if 'model_weights' in f else f  # save_weights() files have no wrapper
        for lname in [_s(n) for n in g.attrs['layer_names']]:
            lg = g[lname]
            wnames = [_s(n) for n in lg.attrs.get('weight_names', [])]
            if not wnames:
                continue
            ws = {}
            for wn in wnames:
                short = wn.split('/')[-1].split(':')[0]
                ws[short] = np.asarray(lg[wn], dtype=np.float32)
            if set(ws) == {'kernel', 'bias'}:
                out.append(('dense', ws))
            elif set(ws) == set(BN_KEYS):
                out.append(('bn', ws))
            else:
                raise ValueError(f'{path}: layer {lname} has unexpected weights {sorted(ws)}')
    return out


def convert(h5_path, scaler_npz):
    layers = read_layers(h5_path)
    kinds = [k for k, _ in layers]
    want = ['dense', 'bn'] * 5 + ['dense']
    if kinds != want:
        raise ValueError(f'{h5_path}: weighted layers {kinds}, expected {want} (train_speech_model.py:55-90)')
    out = {}
    for i in range(5):
        d, bn = layers[2 * i][1], layers[2 * i + 1][1]
        out[f'dense_{i}/kernel'] = d['kernel']
        out[f'dense_{i}/bias'] = d['bias']
        for k in BN_KEYS:
            out[f'batch_normalization_{i}/{k}'] = bn[k]
    out['dense_5/kernel'] = layers[10][1]['kernel']
    out['dense_5/bias'] = layers[10][1]['bias']
    for i in range(6):
        k = out[f'dense_{i}/kernel']
        if k.shape != (DIMS[i], DIMS[i + 1]):
            raise ValueError(f'dense_{i}/kernel has shape {k.shape}, expected {(DIMS[i], DIMS[i + 1])}')
    if scaler_npz:
        with np.load(scaler_npz, allow_pickle=False) as z:
            out['scaler/mean_'] = np.asarray(z['mean_'], dtype=np.float32)
            out['scaler/scale_'] = np.asarray(z['scale_'], dtype=np.float32)
    else:  # the reference runs without a scaler when none was saved (speech_inference.py:24-34)
        out['scaler/mean_'] = np.zeros(56, np.float32)
        out['scaler/scale_'] = np.ones(56, np.float32)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split('\n')[0])
    ap.add_argument('h5')
    ap.add_argument('--scaler', default=None, help='npz with mean_ and scale_ (see module docstring)')
    ap.add_argument('-o', '--out', required=True)
    a = ap.parse_args(argv)
    w = convert(a.h5, a.scaler)
    np.savez(a.out, **w)
    print(f'wrote {a.out}: {len(w)} arrays', file=sys.stderr)


if __name__ == '__main__':
    main()
