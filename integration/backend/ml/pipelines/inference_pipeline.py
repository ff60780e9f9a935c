"""Drop-in for backend/ml/pipelines/inference_pipeline.py (what backend/api/views.py:12-13
imports), served by mmdx.  The relative imports below are the reference module's own
(inference_pipeline.py:25-29)."""
from . import _mmdx_path  # noqa: F401

from .training_pipeline import ImageEncoderCNN  # noqa: F401
from .training_pipeline import TextEncoderTransformer  # noqa: F401
from .training_pipeline import FusionTransformerModel  # noqa: F401
from .training_pipeline import image_transfom_into_tensor, tokenize_patient_details  # noqa: F401
from .training_pipeline import parse_s3_url, get_image_from_s3  # noqa: F401

from mmdx.inference_pipeline import (  # noqa: F401
    inference, inference_tests, latest_version, load_model_bundle,
    load_model_from_hopsworks_model_registry, save_model_bundle)
