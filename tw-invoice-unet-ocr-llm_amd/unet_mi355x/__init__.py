"""MI355X-native UNet forward path (drop-in for tingyu-c/TW-invoice-unet-ocr-llm's
unet_model.UNet / inference.run_unet).  See DESIGN.md at the repository root."""
from .model import UNet, DoubleConv  # noqa: F401

__all__ = ["UNet", "DoubleConv"]
