"""Drop-in replacement module for the reference ``unet_model.py``.

Put this directory on sys.path (or copy this shim next to the app) and
``from unet_model import UNet`` (app_camera.py / inference.py:4) gets the MI355X path.
"""
from unet_mi355x.model import DoubleConv, UNet  # noqa: F401
