"""Constants mirrored from the reference's config.py (constants that feed the hot path only).

Reference: config.py:39-44 (model paths), :53 (EMOTIONS order — drives every
argmax -> label mapping), :57-59 (audio), :62 (MAX_TEXT_LENGTH), :65 (IMAGE_SIZE).
Web/session/database settings are out of scope.
"""
import os


class Config:
    # Model paths (config.py:39-44); relative to CWD exactly like the reference.
    SPEECH_MODEL_PATH = os.environ.get('SPEECH_MODEL_PATH', 'models/speech_model.h5')
    SPEECH_SCALER_PATH = os.environ.get('SPEECH_SCALER_PATH', 'models/speech_scaler.pkl')
    TEXT_MODEL_PATH = os.environ.get('TEXT_MODEL_PATH', 'models/text_model.h5')
    IMAGE_MODEL_PATH = os.environ.get('IMAGE_MODEL_PATH', 'models/image_model.h5')
    FUSION_MODEL_PATH = os.environ.get('FUSION_MODEL_PATH', 'models/fusion_model.pkl')
    BERT_MODEL_PATH = os.environ.get('BERT_MODEL_PATH', 'models/bert_model')

    # Labels (config.py:53-54)
    EMOTIONS = ['happy', 'sad', 'angry', 'fear', 'disgust', 'surprise', 'neutral']
    NUM_EMOTIONS = 7

    # Audio settings (config.py:57-59)
    SAMPLE_RATE = 22050
    AUDIO_DURATION = 3
    N_MFCC = 40

    # Text settings (config.py:62)
    MAX_TEXT_LENGTH = 128

    # Image settings (config.py:65)
    IMAGE_SIZE = (224, 224)

    # Build-only: seed for deterministic synthetic weights when no trained
    # checkpoint exists (the reference ships none: .gitignore:25-30).
    SYNTHETIC_SEED = os.environ.get('MEC_SYNTHETIC_SEED')

    # Build-only: arithmetic of the drop-in classes' BERT / ResNet50 / MobileNetV2 forwards.
    # 'fp32' (default) is the reference's own (inference/text_inference.py:91-93,
    # inference/image_inference.py:116-118); 'f16' is the fast path (f16 MFMA operands, fp32
    # accumulation; probs within 1e-3). Speech, fusion and audio are fp32 either way.
    PRECISION = os.environ.get('MEC_PRECISION', 'fp32')
