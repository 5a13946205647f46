"""keyhunt_amd -- MI355X-native engine for keyhunt's secp256k1 key-search hot path.

The compute lives in HIP kernels for gfx950 behind the C ABI in include/kh_gpu.h
(keyhunt_amd/lib/libkh_gpu.so); `keyhunt_amd.engine` is its ctypes binding and
keyhunt_amd/bin/keyhunt-amd the C++ command-line host with the reference's -m/-f/-r/-b/-k flags.
"""
from .engine import (Engine, KhError, build, device_count, header_symbols, lib, LIB_PATH,  # noqa: F401
                     KH_MODE_ADDRESS, KH_MODE_XPOINT, KH_MODE_ETH, KH_MODE_ENDO, KH_SEARCH_COMPRESS, KH_SEARCH_UNCOMPRESS, KH_SEARCH_BOTH,
                     KH_KIND_02, KH_KIND_03, KH_KIND_04, KH_KIND_XPOINT, KH_KIND_ETH, KH_KIND_ENDO1, KH_KIND_ENDO2, KH_KIND_NEGY, ORDER_N, KH_LAYER1_REFERENCE,
                     KH_LAYER1_BLOCKED)

__all__ = ["Engine", "KhError", "build", "device_count", "header_symbols", "lib", "LIB_PATH"]
