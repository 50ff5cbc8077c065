"""ORACLE (test infrastructure only): speech DNN with Keras inference semantics, fp32.

Restates
  scaler.transform(x)        inference/speech_inference.py:66-67, :86-87
                             (sklearn StandardScaler: (x - mean_) / scale_)
  model.predict(x)           inference/speech_inference.py:69, :103 on the Sequential of
                             model_training/train_speech_model.py:55-90:
                             5 x [Dense -> BatchNormalization(eps=1e-3) -> ReLU -> Dropout]
                             -> Dense(7, softmax). Dropout is identity at inference.
  layers[-3].output          inference/speech_inference.py:93-97: layers[-1]=Dense7,
                             layers[-2]=Dropout, layers[-3]=block-5 Activation (ReLU) -> 64-d.
BatchNormalization follows tf.nn.batch_normalization's formula
  inv = rsqrt(var + eps) * gamma ; y = x * inv + (beta - mean * inv).
TensorFlow is absent here, so this restatement is parity-unpinned (oracle/__init__.py).
"""
import numpy as np

EPS = np.float32(1e-3)  # keras.layers.BatchNormalization default epsilon


def softmax(z: np.ndarray) -> np.ndarray:
    z = z - z.max(axis=-1, keepdims=True)
    e = np.exp(z)
    return (e / e.sum(axis=-1, keepdims=True)).astype(np.float32)


def forward(w, x_raw: np.ndarray):
    """x_raw f32 [B,56] (pre-scaler) -> (feat64 [B,64], logits [B,7], probs [B,7])."""
    x = (np.asarray(x_raw, np.float32) - w['scaler/mean_']) / w['scaler/scale_']
    for i in range(5):
        y = x @ w[f'dense_{i}/kernel'] + w[f'dense_{i}/bias']
        g = w[f'batch_normalization_{i}/gamma']
        inv = (np.float32(1.0) / np.sqrt(w[f'batch_normalization_{i}/moving_variance'] + EPS)) * g
        y = y * inv + (w[f'batch_normalization_{i}/beta'] - w[f'batch_normalization_{i}/moving_mean'] * inv)
        x = np.maximum(y, np.float32(0.0)).astype(np.float32)
    feat = x
    logits = (feat @ w['dense_5/kernel'] + w['dense_5/bias']).astype(np.float32)
    return feat, logits, softmax(logits)
