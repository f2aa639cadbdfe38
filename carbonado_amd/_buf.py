"""Zero-copy views of host buffers for the C-ABI calls."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .error import status_to_error


def as_u8(data) -> np.ndarray:
    """A contiguous uint8 view of bytes / bytearray / memoryview / ndarray."""
    if isinstance(data, np.ndarray):
        a = data.reshape(-1).view(np.uint8)
        return np.ascontiguousarray(a)
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data if a.size else 0)


def check(status: int) -> None:
    if status != 0:
        detail = ""
        if status in (100, 101):
            raw = _lib.lib().chip_last_device_error()
            detail = raw.decode() if raw else ""
        raise status_to_error(status, detail)
