"""GGUF container and ggml block-format constants (GGUF v3).

Upstream format facts (SURVEY §2.3 "Quantisation formats that must be exact");
the reference reaches these through llama-cpp-python (reference
docker/Dockerfile.base:30-32, api.py:24-28).
"""
from enum import IntEnum

GGUF_MAGIC = 0x46554747  # b"GGUF" little-endian
GGUF_VERSION = 3
GGUF_DEFAULT_ALIGNMENT = 32


class GGUFValueType(IntEnum):
    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


class GGMLType(IntEnum):
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    BF16 = 30


# (block size in weights, bytes per block)
GGML_BLOCK = {
    GGMLType.F32: (1, 4),
    GGMLType.F16: (1, 2),
    GGMLType.BF16: (1, 2),
    GGMLType.Q8_0: (32, 34),
    GGMLType.Q4_K: (256, 144),
    GGMLType.Q5_K: (256, 176),
    GGMLType.Q6_K: (256, 210),
}

QK_K = 256

# llama_ftype values written to general.file_type
FTYPE_ALL_F32 = 0
FTYPE_MOSTLY_F16 = 1
FTYPE_MOSTLY_Q8_0 = 7
FTYPE_MOSTLY_Q4_K_M = 15
FTYPE_MOSTLY_Q5_K_M = 17
FTYPE_MOSTLY_Q6_K = 18

# llama vocab token types
TOKEN_TYPE_NORMAL = 1
TOKEN_TYPE_UNKNOWN = 2
TOKEN_TYPE_CONTROL = 3
TOKEN_TYPE_USER_DEFINED = 4
TOKEN_TYPE_UNUSED = 5
TOKEN_TYPE_BYTE = 6


def tensor_nbytes(ggml_type: int, n_elements: int) -> int:
    bs, bb = GGML_BLOCK[GGMLType(ggml_type)]
    assert n_elements % bs == 0, (ggml_type, n_elements)
    return n_elements // bs * bb
