"""Drop-in replacement module for the reference ``inference.py`` (``from inference import
run_unet``, app_camera.py:16)."""
from unet_mi355x.inference import (DEVICE, FIELDS, IMG_SIZE, load_model, preprocess,  # noqa: F401
                                   run_unet)
