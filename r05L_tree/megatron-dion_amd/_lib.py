"""ctypes binding of the C ABI in include/dion_codec.h (libdion_codec.so).

The library is built in-tree by `python __graft_entry__.py` (hipcc, gfx950) and
must be present: there is no CPU or PyTorch fallback for the codec.  A missing
or stale library raises `DionLibraryError` at first use.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(HERE, "csrc", "libdion_codec.so")


def _lib_path() -> str:
    """The in-tree library, unless a kernel-variant A/B run names another build of the same ABI.

    A variant needs BOTH `DION_LIB_PATH` and `DION_DEV_ALLOW_LIB_PATH=1` (a dev-only switch
    that no product path, test, smoke() or bench.py sets), and its use is announced on
    stderr: an environment variable alone can never swap the product's kernels silently."""
    alt = os.environ.get("DION_LIB_PATH")
    if not alt:
        return DEFAULT_LIB_PATH
    if os.environ.get("DION_DEV_ALLOW_LIB_PATH") != "1":
        raise RuntimeError(f"[DION_LIB_PATH_NOT_ALLOWED] DION_LIB_PATH={alt!r} is a dev-only override; "
                           "set DION_DEV_ALLOW_LIB_PATH=1 to load a variant build, or unset DION_LIB_PATH")
    print(f"[dion] WARNING: loading codec variant {alt} (DION_LIB_PATH), not {DEFAULT_LIB_PATH}",
          file=sys.stderr, flush=True)
    return alt


LIB_PATH = _lib_path()
SOURCES = (os.path.join(HERE, "csrc"), os.path.join(os.path.dirname(HERE), "include"))


def source_build_id(roots=SOURCES) -> str | None:
    """SHA-256 (16 hex digits) over the codec's sources: csrc/dion_codec.hip, csrc/*.hpp and
    include/dion_codec.h, by file name then bytes, sorted by name.  __graft_entry__.build()
    compiles it in as DION_BUILD_ID; load() compares.  None when the sources are absent."""
    files = []
    for root in roots:
        if not os.path.isdir(root):
            continue
        for name in os.listdir(root):
            if name == "dion_codec.hip" or name.endswith(".hpp") or name == "dion_codec.h":
                files.append((name, os.path.join(root, name)))
    if not any(n == "dion_codec.hip" for n, _ in files):
        return None
    h = hashlib.sha256()
    for name, path in sorted(files):
        h.update(name.encode())
        h.update(b"\0")
        with open(path, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
ABI_VERSION = 15

DION_OK = 0
DION_E_INVALID = -1
DION_E_UNSUPPORTED = -2
DION_E_LAUNCH = -3
DION_E_WORKSPACE = -4

DTYPE_NONE = 0
DTYPE_F32 = 1
DTYPE_BF16 = 2

OP_PROJECT_P = 1
OP_ORTHONORMALIZE = 2
OP_PROJECT_R = 3
OP_FIXUP_COLNORM = 4
OP_PROJECT_P_EF = 5
OP_EF_APPLY = 6
OP_GRAD_SUM_SQ = 7
OP_DORTHO = 8
OP_PSPLIT = 9

# every symbol include/dion_codec.h declares
EXPORTED = (
    "dion_abi_version",
    "dion_build_id",
    "dion_last_error",
    "dion_workspace_bytes",
    "dion_project_p",
    "dion_project_p_ef",
    "dion_orthonormalize",
    "dion_orthonormalize_fused",
    "dion_dortho_sketch",
    "dion_dortho_qr_inv",
    "dion_dortho_apply",
    "dion_dortho_gram",
    "dion_dortho_chol_inv",
    "dion_project_r",
    "dion_project_r_split",
    "dion_project_r_fixup",
    "dion_fixup_colnorm",
    "dion_fixup_colsum",
    "dion_colnorm_apply",
    "dion_ef_apply",
    "dion_round_bf16",
    "dion_grad_sum_sq",
    "dion_elementwise_adamw",
    "dion_elementwise_lion",
)


class DionLibraryError(RuntimeError):
    """A failed C-ABI call; `code` is its DION_E_* return code."""
    code = None


class DionUnsupportedError(DionLibraryError):
    """DION_E_UNSUPPORTED: the call refused the shape / layout before enqueuing any work
    (include/dion_codec.h), so the caller may take another path."""


class DionBatchDesc(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int32),
        ("m", ctypes.c_int32),
        ("n", ctypes.c_int32),
        ("r", ctypes.c_int32),
        ("transposed", ctypes.c_int32),
        ("g_dtype", ctypes.c_int32),
        ("m_dtype", ctypes.c_int32),
        ("w_dtype", ctypes.c_int32),
        ("ld_g", ctypes.c_int64),
        ("ld_m", ctypes.c_int64),
        ("ld_w", ctypes.c_int64),
    ]


class DionPendingEF(ctypes.Structure):
    _fields_ = [("P", ctypes.POINTER(ctypes.c_void_p)), ("R", ctypes.POINTER(ctypes.c_void_p)),
                ("alpha", ctypes.c_float)]


_P = ctypes.c_void_p
_PP = ctypes.POINTER(ctypes.c_void_p)
_DESC = ctypes.POINTER(DionBatchDesc)

_SIGNATURES = {
    "dion_abi_version": ([], ctypes.c_int),
    "dion_build_id": ([], ctypes.c_char_p),
    "dion_last_error": ([], ctypes.c_char_p),
    "dion_workspace_bytes": ([_DESC, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "dion_project_p": ([_DESC, _PP, _PP, _PP, _P, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_project_p_ef": ([_DESC, _PP, _PP, _PP, _P, _P, ctypes.POINTER(DionPendingEF), _P, ctypes.c_size_t, _P],
                          ctypes.c_int),
    "dion_orthonormalize": ([_DESC, _P, _P, ctypes.c_uint64, ctypes.c_float, _P, ctypes.c_size_t, _P],
                            ctypes.c_int),
    "dion_project_r": ([_DESC, _PP, _P, _P, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_orthonormalize_fused": ([_DESC, _P, _P, ctypes.c_uint64, ctypes.c_float, _P, _P, _P, ctypes.c_size_t, _P],
                                  ctypes.c_int),
    "dion_project_r_split": ([_DESC, _PP, _P, _P, _P, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_project_r_fixup": ([_DESC, _PP, _P, _P, _P, _P, _PP, _P, ctypes.c_float, _P, ctypes.c_size_t, _P],
                             ctypes.c_int),
    "dion_fixup_colnorm": ([_DESC, _P, _P, _PP, _P, ctypes.c_float, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_fixup_colsum": ([_DESC, _P, _P, _PP, _P, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_colnorm_apply": ([_DESC, _P, _PP, _P, ctypes.c_float, _P], ctypes.c_int),
    "dion_ef_apply": ([_DESC, _PP, _PP, _P, _P, _PP, _P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                       ctypes.c_double, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_dortho_sketch": ([_DESC, _P, _P, ctypes.c_uint64, ctypes.c_int64, ctypes.c_float, _P, _P, ctypes.c_size_t,
                            _P], ctypes.c_int),
    "dion_dortho_qr_inv": ([ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P], ctypes.c_int),
    "dion_dortho_apply": ([_DESC, _P, _P, _P, _P], ctypes.c_int),
    "dion_dortho_gram": ([_DESC, _P, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_dortho_chol_inv": ([ctypes.c_int32, ctypes.c_int32, _P, _P, _P], ctypes.c_int),
    "dion_round_bf16": ([_P, ctypes.c_int64, _P], ctypes.c_int),
    "dion_grad_sum_sq": ([_DESC, _PP, _P, _P, ctypes.c_size_t, _P], ctypes.c_int),
    "dion_elementwise_adamw": ([ctypes.c_int32, _P, _PP, _PP, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _PP, _PP,
                                ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int32,
                                _P], ctypes.c_int),
    "dion_elementwise_lion": ([ctypes.c_int32, _P, _PP, _PP, ctypes.c_int32, ctypes.c_int32, _PP, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, ctypes.c_double, _P], ctypes.c_int),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load (once) and return the codec library; raise if it is missing or stale."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise DionLibraryError(
            f"[DION_HIP_LIBRARY_MISSING] {path} not found; build it with "
            "`python __graft_entry__.py` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (args, res) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    ver = lib.dion_abi_version()
    if ver != ABI_VERSION:
        raise DionLibraryError(f"[DION_HIP_ABI_MISMATCH] library ABI {ver}, expected {ABI_VERSION}")
    want = source_build_id()
    got = lib.dion_build_id().decode("ascii", "replace")
    if path == DEFAULT_LIB_PATH and want is not None and got != want:
        raise DionLibraryError(
            f"[DION_HIP_LIBRARY_STALE] {path} was built from sources {got}, the tree holds {want}; rebuild it "
            "with `python __graft_entry__.py`")
    if path == LIB_PATH:
        _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != DION_OK:
        msg = load().dion_last_error().decode("utf-8", "replace")
        cls = DionUnsupportedError if rc == DION_E_UNSUPPORTED else DionLibraryError
        err = cls(f"[DION_HIP_ERROR] {what} failed ({rc}): {msg}")
        err.code = rc
        raise err
