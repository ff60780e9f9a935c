"""Drop-in for backend/ml/pipelines/training_pipeline.py: every name the reference's callers
import from it (inference_pipeline.py:25-29, run_daily_training_pipeline.py:2), served by
mmdx on the MI355X.  Copy this directory over backend/ml/pipelines/ (or keep it on
sys.path); set MMDX_HOME to the mmdx checkout."""
from . import _mmdx_path  # noqa: F401

from mmdx.training_pipeline import *  # noqa: F401,F403
from mmdx.training_pipeline import (  # noqa: F401
    BCEWithLogitsLoss, CXR_ImageDataset, DISEASES, FusionTransformerModel, IMG_SIZE,
    ImageEncoderCNN, TextEncoderTransformer, construct_input_label_pairs_for_image_encoder_dataset,
    get_image_from_s3, image_transfom_into_tensor, load_features_labels_from_feature_store,
    parse_s3_url, save_model_to_hopsworks_model_registry, tokenize_patient_details,
    training_tests)
