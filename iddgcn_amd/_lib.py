"""ctypes binding of libiddgcn_hip.so (C-ABI declared in include/iddgcn.h, iddgcn_graph.h,
iddgcn_similarity.h and iddgcn_sampling.h).

The product path has no CPU fallback: if the shared library is missing, was
built for another ABI version or from other sources than the tree beside it
(the source digest compiled into it, _srchash.py), :func:`lib` raises immediately.
"""
import ctypes
import os

from . import _srchash

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(_HERE, "libiddgcn_hip.so")
LIB_PATH = PRODUCT_LIB
# a build variant of the same source (tools/ A/B timing, built with extra -D flags: no source digest check); the
# product loads PRODUCT_LIB
if os.environ.get("IDDGCN_LIB"):
    LIB_PATH = os.environ["IDDGCN_LIB"]
ABI_VERSION = 12
ROWGEMM_BATCH = 25          # IDDGCN_ROWGEMM_BATCH: entries per iddgcn_rowgemm_batched_f32 call

ACT_NONE, ACT_SIGMOID, ACT_DSIGMOID = 0, 1, 2
GEMM_EXACT_F32, GEMM_SPLIT_F16, GEMM_F32_4CHAIN, GEMM_BF16X3, GEMM_BF16 = 0, 1, 2, 3, 4
PLANES_A, PLANES_C, PLANES_AUX = 1, 2, 4          # iddgcn_rowgemm_t.planes (pre-split edge tables, ABI 4)

vp = ctypes.c_void_p
ci = ctypes.c_int
cll = ctypes.c_longlong
cf = ctypes.c_float


class RowGemmArgs(ctypes.Structure):
    """Mirror of iddgcn_rowgemm_t."""
    _fields_ = [
        ("M", ci), ("D", ci),
        ("A", vp), ("a_idx", vp),
        ("B", vp), ("b_trans", ci),
        ("C", vp), ("accumulate", ci),
        ("R", ci),
        ("coef", vp), ("coef_idx", vp),
        ("V", vp), ("v_idx", vp),
        ("v_rel_stride", cll), ("v_row_stride", cll),
        ("act", ci), ("aux", vp),
        ("planes", ci),
        ("precision", ci),     # ABI 6/7: operand precision per call (GEMM_EXACT_F32 / F32_4CHAIN / SPLIT_F16 / BF16X3)
    ]


class TnArgs(ctypes.Structure):
    """Mirror of iddgcn_tn_t (ABI 5)."""
    _fields_ = [("M", cll), ("A", vp), ("B", vp), ("C", vp), ("accumulate", ci)]


TN_BATCH = 4


# name -> (restype, argtypes)
SIGNATURES = {
    "iddgcn_abi_version": (ci, []),
    "iddgcn_spmm_csr_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, ci]),
    "iddgcn_sddmm_csr_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp]),
    "iddgcn_rowgemm_f32": (ci, [vp, ctypes.POINTER(RowGemmArgs)]),
    "iddgcn_gemm_tn_blocks": (ci, [cll, ci]),
    "iddgcn_gemm_tn_f32": (ci, [vp, cll, ci, vp, vp, vp, ci, vp, ci, ci]),
    "iddgcn_rowgemm_batched_f32": (ci, [vp, ctypes.POINTER(RowGemmArgs), ci]),
    "iddgcn_rowgemm_kernel_id": (ci, [ctypes.POINTER(RowGemmArgs)]),
    "iddgcn_adam_table_f32": (ci, [vp, cll, vp, vp, vp, vp, vp, vp, cf, cf, cf, ci]),
    "iddgcn_step_advance": (ci, [vp, vp, vp, vp]),
    "iddgcn_gemm_tn_narrow_blocks": (ci, [cll]),
    "iddgcn_gemm_tn_narrow_f32": (ci, [vp, cll, ci, ci, vp, vp, vp, ci, vp, vp, ci]),
    "iddgcn_alpha_fwd_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, vp]),
    "iddgcn_combine_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, cll, vp]),
    "iddgcn_distmult_blocks": (ci, [cll]),
    "iddgcn_distmult_bce_f32": (ci, [vp, cll, ci, ci, vp, vp, vp, vp, vp, vp, vp, cf, vp, vp, vp, vp, vp, vp, ci]),
    "iddgcn_distmult_bce_heads_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp, cf, vp, vp, vp, vp, vp, vp,
                                           vp, ci]),
    "iddgcn_seg_gather_reduce_f32": (ci, [vp, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp]),
    "iddgcn_tail_seg_reduce_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, cll, vp, cll, vp, vp]),
    "iddgcn_head_bwd_node_f32": (ci, [vp, ci, ci, ci, vp, vp, cll, vp, vp, vp, vp, vp, vp, vp, cll, vp, vp]),
    "iddgcn_head_wsum_f32": (ci, [vp, ci, ci, vp, vp, vp, vp]),
    "iddgcn_gather_rows_f32": (ci, [vp, cll, ci, vp, vp, vp]),
    "iddgcn_reduce_slabs_f32": (ci, [vp, ci, cll, vp, vp, ci, cf]),
    "iddgcn_adam_f32": (ci, [vp, cll, vp, vp, vp, vp, cf, cf, cf, cf, ci]),
    # bf16-feature mode
    "iddgcn_rowgemm_bf16": (ci, [vp, ctypes.POINTER(RowGemmArgs)]),
    "iddgcn_gemm_tn_bf16": (ci, [vp, cll, ci, vp, vp, vp, ci, vp, ci]),
    "iddgcn_sigma_tn_ranges": (ci, [cll]),
    "iddgcn_sigma_tn_bf16": (ci, [vp, cll, ci, vp, vp, vp, vp, cll, vp, ci]),
    "iddgcn_sigma_tn_f32": (ci, [vp, cll, ci, vp, vp, vp, vp, cll, vp, ci]),
    "iddgcn_combine_bf16": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, cll, vp]),
    "iddgcn_combine_planes_f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, cll, vp]),
    "iddgcn_gemm_tn_planes_f32": (ci, [vp, cll, ci, vp, vp, vp, ci, vp, ci]),
    "iddgcn_gemm_tn_batched_f32": (ci, [vp, ci, ctypes.POINTER(TnArgs), ci, vp, cll, ci]),
    "iddgcn_distmult_bce_bf16": (ci, [vp, cll, ci, ci, vp, vp, vp, vp, vp, vp, vp, cf, vp, vp, vp, vp, vp, vp, ci]),
    "iddgcn_distmult_bce_heads_bf16": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp, cf, vp, vp, vp, vp, vp, vp,
                                            vp, ci]),
    "iddgcn_tail_seg_reduce_bf16": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp, cll, vp, cll, vp, vp]),
    "iddgcn_tail_seg_reduce_head_bf16": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, cll, vp, cll, vp, vp, vp, vp, vp]),
    "iddgcn_head_dz_f32": (ci, [vp, ci, ci, vp, vp, vp, vp, vp, vp, vp]),
    # include/iddgcn_graph.h
    "iddgcn_radix_sort_workspace": (cll, [cll, ci]),
    "iddgcn_radix_sort_pairs": (ci, [vp, cll, ci, ci, vp, vp, vp, vp, vp, cll]),
    "iddgcn_adjacency_workspace": (cll, [cll, ci, ci]),
    "iddgcn_build_adjacency": (ci, [vp, cll, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, cll]),
    "iddgcn_scored_edges_workspace": (cll, [cll, ci]),
    "iddgcn_build_scored_edges": (ci, [vp, cll, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, cll]),
    # include/iddgcn_sampling.h
    "iddgcn_randint_mask": (ctypes.c_uint32, [ctypes.c_uint32]),
    "iddgcn_mt19937_seed": (ci, [vp, ctypes.c_uint32, vp]),
    "iddgcn_mt19937_generate": (ci, [vp, vp, cll, vp]),
    "iddgcn_accept_chunks": (cll, [cll]),
    "iddgcn_masked_accept": (ci, [vp, vp, cll, ctypes.c_uint32, cll, vp, vp, vp]),
    "iddgcn_assemble_negatives": (ci, [vp, cll, vp, vp, vp, vp]),
    # include/iddgcn_similarity.h
    "iddgcn_similarity_workspace": (cll, [ci, ci]),
    "iddgcn_similarity_pairs": (ci, [vp, ci, ci, vp, ctypes.c_double, vp, cll, vp, cll, vp, vp, cll]),
    "iddgcn_similarity_triples": (ci, [vp, cll, ci, ci, cll, vp, vp]),
}

_lib = None


class IddgcnError(RuntimeError):
    pass


def exported_symbols():
    return list(SIGNATURES)


class StaleLibraryError(IddgcnError):
    pass


def library_source_sha256(lib):
    """The source digest compiled into a loaded library (iddgcn_source_sha256), or None if it exports none."""
    try:
        fn = lib.iddgcn_source_sha256
    except AttributeError:
        return None
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    return fn().decode()


def load(path=LIB_PATH, check_source=None):
    """Load the library and bind every symbol of include/*.h (no GPU call).  ``check_source`` (default: for the
    product library) compares the digest of the sources the library was built from with the tree's (_srchash) and
    raises StaleLibraryError on a mismatch."""
    if not os.path.exists(path):
        raise IddgcnError(
            f"libiddgcn_hip.so not found at {path}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback for the IDDGCN hot path.")
    lib = ctypes.CDLL(path)
    lib.iddgcn_abi_version.restype = ci
    v = lib.iddgcn_abi_version()
    if v != ABI_VERSION:
        raise IddgcnError(f"libiddgcn_hip ABI version {v}, expected {ABI_VERSION}")
    if check_source is None:
        check_source = os.path.abspath(path) == PRODUCT_LIB and not os.environ.get("IDDGCN_LIB")
    if check_source:
        built, tree = library_source_sha256(lib), _srchash.source_sha256()
        if built != tree:
            raise StaleLibraryError(
                f"{path} was built from other sources (digest {built}) than this tree's ({tree}): rebuild it with "
                "`python -c 'import __graft_entry__ as g; g.build()'`")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    global _lib
    if _lib is None:
        _lib = load()
    return _lib


def check(rc, what):
    if rc != 0:
        kind = {-1: "unsupported feature width D", -2: "unsupported relation count R",
                -3: "invalid argument"}.get(rc, f"HIP error {rc}")
        raise IddgcnError(f"{what} failed: {kind}")
