"""mmdx — MI355X-native multimodal diagnosis hot path (import name of this package).

The directory name is `multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd`;
`import mmdx` (repo-root shim `mmdx.py`) loads it.  Public surface mirrors
backend/ml/pipelines/{training,inference}_pipeline.py of the reference.
"""
from . import _lib  # noqa: F401  (lazy: the .so loads on first kernel call)
from .training_pipeline import (  # noqa: F401
    BCEWithLogitsLoss, DISEASES, FusionTransformerModel, IMG_SIZE, ImageEncoderCNN,
    TextEncoderTransformer, get_compute_dtype, image_transfom_into_tensor,
    set_compute_dtype, tokenize_patient_details)
from .optim import AdamW, clip_grad_norm_  # noqa: F401
from .amp import GradScaler  # noqa: F401
from .preprocess import preprocess_batch  # noqa: F401

__version__ = "0.1.0"
