"""Utilities: image I/O, synthetic frames, logging."""
from .io import (read_image, write_image, decode_pnm, encode_pnm, decode_jpeg, encode_jpeg,  # noqa: F401
                 read_image_device, write_image_device)
from .synthetic import synthetic_image, synthetic_rows  # noqa: F401
from .log import get_logger  # noqa: F401
