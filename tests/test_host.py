"""Host logic of the product path (no GPU): graph build, layouts, C-ABI exports."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from iddgcn_amd import _lib
from iddgcn_amd.graph import DeviceAdjacency, ScoredEdges, get_adj_mats
from iddgcn_amd.utils import generate_reverse_triplets, get_y_true, synthetic_graph
from oracle import ref_utils
from tests.conftest import ROOT


def header_symbols():
    import glob
    src = "".join(open(f).read() for f in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    return sorted(set(re.findall(r"^\s*(?:int|long long|uint32_t)\s+(iddgcn_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()          # loads the .so, binds all prototypes, checks ABI version (no GPU call)
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} not bound in _lib.SIGNATURES"
    assert lib.iddgcn_abi_version() == _lib.ABI_VERSION


def test_library_is_tied_to_its_sources(tmp_path):
    """The product library carries the digest of the sources it was built from (iddgcn_source_sha256, ABI 12) and
    it is this tree's; a library whose digest differs (a stale build at the same ABI) is refused by the loader."""
    import subprocess
    from iddgcn_amd import _srchash
    lib = _lib.load()
    assert _lib.library_source_sha256(lib) == _srchash.source_sha256()
    files = _srchash.source_files()
    assert "iddgcn_amd/csrc/iddgcn_hip.hip" in files and "include/iddgcn.h" in files
    assert "iddgcn_amd/csrc/device_flags.txt" in files
    # a stand-in library at the right ABI but built from other sources
    src = tmp_path / "stale.c"
    src.write_text(f'int iddgcn_abi_version(void) {{ return {_lib.ABI_VERSION}; }}\n'
                   f'const char* iddgcn_source_sha256(void) {{ return "{"0" * 64}"; }}\n')
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    with pytest.raises(_lib.StaleLibraryError):
        _lib.load(str(so), check_source=True)
    # one without any digest is refused as well
    src.write_text(f'int iddgcn_abi_version(void) {{ return {_lib.ABI_VERSION}; }}\n')
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    with pytest.raises(_lib.StaleLibraryError):
        _lib.load(str(so), check_source=True)


_ASM = None


def _library_asm():
    """The gfx950 disassembly of every code object in libiddgcn_hip.so (cached)."""
    global _ASM
    if _ASM is None:
        _ASM = _disassemble()
    return _ASM


def test_library_has_no_packed_fp32_valu():
    """The product library is built without packed-fp32 VALU (iddgcn_amd/csrc/device_flags.txt; DESIGN.md
    §Determinism): disassemble the gfx950 code object of libiddgcn_hip.so and find no v_pk_fma_f32 / v_pk_mul_f32 /
    v_pk_add_f32 / v_pk_mov_b32."""
    asm = _library_asm()
    assert "radix" in asm and "tail_seg_reduce" in asm     # every translation unit's kernels were disassembled
    assert asm.count("s_endpgm") > 50          # the kernels really were disassembled
    bad = sorted(set(re.findall(r"\bv_pk_(?:fma|mul|add)_f32\b", asm)))
    assert not bad, f"packed-fp32 VALU in the product library: {bad}"


def _kernel_bodies(asm, pattern):
    """{symbol: [instruction lines]} of the kernels whose symbol matches ``pattern`` (llvm-objdump -d layout: a
    `<symbol>:` header, then one instruction per line)."""
    out, cur = {}, None
    for line in asm.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1) if re.search(pattern, m.group(1)) else None
            if cur:
                out[cur] = []
            continue
        if cur and line.strip():
            ins = line.split("//")[0].strip()
            if ins:
                out[cur].append(ins)
    return out


def _regs(text):
    """VGPR numbers named in an operand list (v7, v[4:7])."""
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        regs.update(range(int(a), int(b) + 1))
    regs.update(int(x) for x in re.findall(r"\bv(\d+)\b", text))
    return regs


def test_asm_transposed_reads_are_waited_for():
    """the TN kernels issue ds_read_b64_tr_b16 from inline asm (hipcc guards the builtin with a vmcnt(0)
    drain), so the compiler does not know the result arrives late; correctness rests on nothing touching a
    destination register before the tied `s_waitcnt lgkmcnt(0)`.  Walk the machine code of every such kernel: between
    a transposed read and the next lgkmcnt(0) no instruction names one of its destination VGPRs (read, copied, spilled
    or overwritten), and the kernels use no scratch."""
    asm = _library_asm()
    kernels = _kernel_bodies(asm, r"gemm_tn256_b3_kernel|gemm_tn256_bf16t_kernel|sigma_tn_bf16_kernel|sigma_tn_b3_kernel")
    assert len(kernels) >= 5, sorted(kernels)       # both sigma_tn_bf16 forms, the two TNs, the fused bf16x3 pass
    for name, body in kernels.items():
        assert not any(i.startswith("scratch_") for i in body), f"{name}: scratch spill"
        pending, n_tr = {}, 0
        for k, ins in enumerate(body):
            op, _, args = ins.partition(" ")
            if op == "s_waitcnt" and "lgkmcnt(0)" in args:
                pending = {}
                continue
            if op == "ds_read_b64_tr_b16":
                n_tr += 1
                dst, _, addr = args.partition(",")
                hit = _regs(args) & set(pending)
                assert not hit, f"{name}: {ins!r} names pending v{sorted(hit)} (line {k})"
                for r in _regs(dst):
                    pending[r] = k
                continue
            hit = _regs(args) & set(pending)
            assert not hit, f"{name}: {ins!r} at line {k} names v{sorted(hit)} before the lgkmcnt(0) of the transposed " \
                            f"read at line {min(pending[r] for r in hit)}"
        assert n_tr > 0, name


def _disassemble():
    import subprocess
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "llvm-objdump")):
        pytest.skip("no ROCm llvm tools")
    asm = ""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(llvm, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, _lib.LIB_PATH,
                        os.path.join(d, "stripped.so")], check=True, capture_output=True)
        blob = open(fat, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), blob)]
        assert len(starts) >= 4, "one offload bundle per source file"
        for i, a in enumerate(starts):         # one bundle per translation unit, concatenated by the link
            part, dev = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"b{i}.o")
            open(part, "wb").write(blob[a:starts[i + 1] if i + 1 < len(starts) else len(blob)])
            subprocess.run([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + part,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + dev], check=True,
                           capture_output=True)
            asm += subprocess.run([os.path.join(llvm, "llvm-objdump"), "-d", dev], check=True, capture_output=True,
                                  text=True).stdout
    return asm


def test_block_helpers_are_pure_host():
    lib = _lib.lib()
    assert lib.iddgcn_gemm_tn_blocks(4_000_000, 256) == 256
    assert lib.iddgcn_gemm_tn_blocks(10, 64) == 1
    assert lib.iddgcn_distmult_blocks(1) == 1


def test_invalid_args_rejected_before_launch():
    lib = _lib.lib()
    # D=48 unsupported, R=9 unsupported: rejected on the host, nothing launched
    assert lib.iddgcn_spmm_csr_f32(None, 1, 4, 48, None, None, None, None, None, 0) == -1
    assert lib.iddgcn_alpha_fwd_f32(None, 4, 64, 9, None, None, None, None, None, None) == -2
    assert lib.iddgcn_adam_f32(None, 4, None, None, None, None, 1.0, .9, .999, 1e-7, 0) == -3
    # the fused sigma' + TN passes accept only their documented operand forms (checked before anything else)
    assert lib.iddgcn_sigma_tn_f32(None, 0, 256, None, None, None, None, 0, None, _lib.GEMM_EXACT_F32) == -3
    assert lib.iddgcn_sigma_tn_f32(None, 0, 256, None, None, None, None, 0, None, 7) == -3
    assert lib.iddgcn_sigma_tn_f32(None, 0, 128, None, None, None, None, 0, None, _lib.GEMM_BF16X3) == -1
    assert lib.iddgcn_sigma_tn_bf16(None, 0, 256, None, None, None, None, 0, None, 7) == -3
    assert lib.iddgcn_sigma_tn_bf16(None, 0, 256, None, None, None, None, 0, None, _lib.GEMM_F32_4CHAIN) == -3


@pytest.mark.parametrize("k", [0, 3])
def test_get_adj_mats_matches_oracle_bit_exact(k, golden):
    d = golden(f"fold{k}_data.npz")
    data = np.concatenate([d["X_train"], d["X_test"]])
    ours = get_adj_mats(data, 845, 4)
    ref = ref_utils.get_adj_coo(data, 845, 4)
    for a, (idx, val) in zip(ours, ref):
        assert a.dense_shape == (1, 845, 845)
        assert np.array_equal(a.indices[:, 0], np.zeros(a.nnz))
        assert np.array_equal(a.indices[:, 1:], idx)
        assert np.array_equal(a.values, val)
    assert [a.nnz for a in get_adj_mats(d["X_train"], 845, 4)] == [1482, 1324, 2346, 32358] if k == 0 else True


def test_empty_relation_placeholder():
    tr = np.array([[0, 0, 1], [1, 0, 0]])
    mats = get_adj_mats(tr, 3, 2)
    assert mats[1].indices.tolist() == [[0, 0, 0]] and mats[1].values.tolist() == [0.0]
    dev = DeviceAdjacency(mats, 3, "cpu")
    assert dev.fwd_val is not None                  # placeholder value 0 is carried
    assert dev.fwd_ptr.tolist() == [0, 1, 2, 2, 2, 3, 3, 3]


def test_device_adjacency_csr_and_transpose():
    pos, _ = synthetic_graph(300, 3, 2000, seed=1)
    mats = get_adj_mats(pos, 300, 3)
    dev = DeviceAdjacency(mats, 300, "cpu")
    ptr, col = dev.fwd_ptr.numpy().reshape(3, 301), dev.fwd_col.numpy()
    for r, a in enumerate(mats):
        rows = np.repeat(np.arange(300), np.diff(ptr[r]))
        cols = col[ptr[r, 0]:ptr[r, -1]]
        assert np.array_equal(np.stack([rows, cols], 1), a.indices[:, 1:])    # CSR order == TF order
    # merged transpose: row c lists r*N+m for every (m, c) in A_r, relation-major then m
    bptr, bcol = dev.bwd_ptr.numpy(), dev.bwd_col.numpy()
    dense = np.zeros((300, 3 * 300))
    for r, a in enumerate(mats):
        dense[a.cols, r * 300 + a.rows] = 1
    got = np.zeros_like(dense)
    for c in range(300):
        seg = bcol[bptr[c]:bptr[c + 1]]
        assert np.all(np.diff(seg) > 0)
        got[c, seg] = 1
    assert np.array_equal(got, dense)


def test_scored_edges_layout():
    rng = np.random.default_rng(0)
    tr = np.stack([rng.integers(0, 50, 400), rng.integers(0, 2, 400), rng.integers(0, 50, 400)], 1)
    lab = rng.random(400).astype(np.float32)
    ed = ScoredEdges(tr, lab, 50, 2, "cpu")
    t, h = ed.t.numpy(), ed.h.numpy()
    assert np.all(np.diff(t) >= 0)                                     # tail-sorted
    assert np.array_equal(tr[ed.order], np.stack([h, ed.r.numpy(), t], 1))
    tptr = ed.tptr.numpy()
    for n in range(50):
        assert np.all(t[tptr[n]:tptr[n + 1]] == n)
    hp, hptr = ed.hperm.numpy(), ed.hptr.numpy()
    for n in range(50):
        seg = hp[hptr[n]:hptr[n + 1]]
        assert np.all(h[seg] == n) and np.all(np.diff(seg) > 0)        # stable
    x = torch.arange(400, dtype=torch.float32)
    assert np.array_equal(ed.unsort(x[torch.as_tensor(ed.order)]).numpy(), x.numpy())
    assert np.array_equal(ed.y.numpy(), lab[ed.order])


def test_index_validation():
    with pytest.raises(_lib.IddgcnError):
        ScoredEdges(np.array([[0, 0, 5]]), None, 5, 1, "cpu")
    with pytest.raises(_lib.IddgcnError):
        ScoredEdges(np.array([[0, 2, 1]]), None, 5, 2, "cpu")
    with pytest.raises(_lib.IddgcnError):
        get_adj_mats(np.array([[0, 0, 7]]), 5, 1)


def test_utils_match_oracle():
    rng = np.random.default_rng(3)
    tr = np.stack([rng.integers(0, 9, 50), rng.integers(0, 2, 50), rng.integers(0, 9, 50)], 1)
    assert np.array_equal(generate_reverse_triplets(tr), ref_utils.generate_reverse_triplets(tr))
    assert np.array_equal(get_y_true(tr[:20], tr), ref_utils.get_y_true(tr[:20], tr))


def test_synthetic_graph_shape_and_rules():
    pos, neg = synthetic_graph(2000, 4, 20000, seed=0)
    assert pos.shape == (20000, 3) and neg.shape == (20000, 3)
    assert np.all(pos[:, 0] != pos[:, 2])
    key = set(map(tuple, pos.tolist()))
    assert len(key) == 20000                                           # unique directed edges
    assert all((t, r, h) in key for h, r, t in pos[:200].tolist())     # reverse-closed
    n_mut = int(round(2000 * 661 / 845))
    resp = pos[pos[:, 1] < 2]
    assert np.all((resp[:, 0] < n_mut) != (resp[:, 2] < n_mut))        # mutation <-> drug
    same = (neg[:, 0] == pos[:, 0]) | (neg[:, 2] == pos[:, 2])
    assert same.all()


def test_model_surface_cpu_only():
    from iddgcn_amd import get_IDDGCN_Model
    m = get_IDDGCN_Model(845, 4, 64, 64, 89, None, 0, 0)
    names = [l.name for l in m.layers]
    assert names == ["entity_embeddings", "iddgcn__layer", "iddgcn__layer_1", "iddgcn__layer_2", "DistMult"]
    shapes = [w.shape for w in m.get_layer("iddgcn__layer").get_weights()]
    assert shapes == [(4, 64, 64), (64, 64), (4,), (64, 4), (4,)]
    assert m.get_layer("DistMult").get_weights()[0].shape == (4, 64)
    w = m.get_layer("entity_embeddings").get_weights()[0]
    assert w.shape == (845, 64) and w.min() >= 0 and w.max() < 1


def test_init_schemes():
    """model.INIT_SCHEMES: the default "tf27" replays TF 2.7's draws (iddgcn_amd/tf_random.py, pinned against the
    bundled weights in tests/test_tf_random.py): the model's weights equal tf_random.reference_init's in the
    reference's creation order, the seeded normal kernel continues its stream (self_kernel is not
    relation_kernels[0]), W_alpha differs per layer, b_alpha = 0; "independent" draws the same distributions from
    numpy.  Both deterministic per seed."""
    from iddgcn_amd import get_IDDGCN_Model
    from iddgcn_amd.tf_random import reference_init
    m = get_IDDGCN_Model(845, 4, 64, 64, 89, None, 0, 0)
    ref = reference_init(845, 4, 64, 89)
    assert np.array_equal(m.get_layer("entity_embeddings").get_weights()[0], ref["E"])
    for l, name in enumerate(("iddgcn__layer", "iddgcn__layer_1", "iddgcn__layer_2"), 1):
        K, S, relw, Wa, ba = m.get_layer(name).get_weights()
        for a, b in ((K, ref[f"K{l}"]), (S, ref[f"S{l}"]), (relw, ref[f"relw{l}"]), (Wa, ref[f"Wa{l}"]),
                     (ba, ref[f"ba{l}"])):
            assert np.array_equal(a, b), (name, a.shape)
    assert np.array_equal(m.get_layer("DistMult").get_weights()[0], ref["rel"])
    K, S = ref["K1"], ref["S1"]
    assert not np.array_equal(S, K[0]) and not np.array_equal(ref["K2"], K)
    assert abs(K.std() - 1.0) < 0.02 and abs(K.mean()) < 0.03
    lim = np.sqrt(6.0 / (64 + 4))
    assert np.abs(ref["Wa1"]).max() <= lim and not np.array_equal(ref["Wa1"], ref["Wa2"])
    again = get_IDDGCN_Model(845, 4, 64, 64, 89, None, 0, 0).get_weights()
    assert all(np.array_equal(a, b) for a, b in zip(m.get_weights(), again))
    ind = get_IDDGCN_Model(845, 4, 64, 64, 89, None, 0, 0, init="independent")
    Ki, Si = ind.get_layer("iddgcn__layer").get_weights()[:2]
    assert not np.array_equal(Si, Ki[0]) and abs(Si.std() - 1.0) < 0.02


def test_load_npz_weights(golden, tmp_path):
    from iddgcn_amd import get_IDDGCN_Model
    m = get_IDDGCN_Model(845, 4, 64, 64, 89, None, 0, 0)
    m.load_weights(os.path.join(ROOT, "tests", "golden", "weights_fold0.npz"))
    g = golden("weights_fold0.npz")
    assert np.array_equal(m.get_layer("entity_embeddings").get_weights()[0], g["E"])
    assert np.array_equal(m.get_layer("iddgcn__layer_2").get_weights()[3], g["Wa3"])
    p = str(tmp_path / "w.npz")
    m.save_weights(p)
    m2 = get_IDDGCN_Model(845, 4, 64, 64, 1, None, 0, 0)
    m2.load_weights(p)
    for a, b in zip(m.get_weights(), m2.get_weights()):
        assert np.array_equal(a, b)


def test_graph_build_workspace_queries_are_pure_host():
    lib = _lib.lib()
    assert lib.iddgcn_radix_sort_workspace(1000, 4) > 1000 * 8
    assert lib.iddgcn_radix_sort_workspace(1000, 8) > lib.iddgcn_radix_sort_workspace(1000, 4)
    assert lib.iddgcn_radix_sort_workspace(1000, 3) < 0
    assert lib.iddgcn_radix_sort_workspace(1 << 31, 4) < 0
    assert lib.iddgcn_adjacency_workspace(37510, 845, 4) > 0
    assert lib.iddgcn_adjacency_workspace(10, 0, 4) < 0
    assert lib.iddgcn_adjacency_workspace(10, 1 << 30, 2) < 0          # R*N >= 2^31
    assert lib.iddgcn_scored_edges_workspace(40316, 845) > 0
    assert lib.iddgcn_scored_edges_workspace(-1, 845) < 0
    # invalid arguments are rejected before any launch (no GPU needed)
    assert lib.iddgcn_radix_sort_pairs(None, 10, 4, 40, None, None, None, None, None, 0) == -3
    assert lib.iddgcn_build_adjacency(None, 10, 0, 4, None, None, None, None, None, None, None, None, None,
                                      None, 0) == -3


def test_rowgemm_precision_is_a_per_call_argument():
    """ABI 6: the GEMM operand precision travels with each call (iddgcn_rowgemm_t.precision, the TN entries'
    `precision`); there is no process-global switch left to race on, and an unknown mode is refused before
    anything is launched."""
    lib = _lib.lib()
    assert not hasattr(lib, "iddgcn_set_gemm_precision") or "iddgcn_set_gemm_precision" not in header_symbols()
    assert "iddgcn_set_gemm_precision" not in _lib.SIGNATURES and "iddgcn_set_rowgemm_path" not in _lib.SIGNATURES
    args = _lib.RowGemmArgs(M=0, D=256, precision=7)
    assert lib.iddgcn_rowgemm_f32(None, args) == -3
    args.precision = _lib.GEMM_SPLIT_F16
    assert lib.iddgcn_rowgemm_f32(None, args) == 0          # M = 0: valid, nothing to do
    assert lib.iddgcn_gemm_tn_f32(None, 32, 256, None, None, None, 1, None, 0, 0) == -3


def test_bf16x3_kernel_selection_is_pure_host():
    """ABI 7: which D = 256 kernel a bf16x3 row GEMM takes (iddgcn_rowgemm_kernel_id, nothing launched, no GPU):
    the column-half bf16x3 kernel (500 + 10 NV + aux + 2 bc) for the plain form, C += A B, the sigma' backward,
    the gathered forward with R = NV <= 2 per-edge coefficients and broadcast V rows (R <= 2); the exact
    kernel's id for every form it does not take (gathered A, accumulate with an activation, coef_idx, R > 2,
    D < 256)."""
    lib = _lib.lib()
    fake = ctypes.c_void_p(16)          # never dereferenced: kernel_id inspects the arguments only

    def kid(**kw):
        a = _lib.RowGemmArgs(M=1000, D=kw.pop("D", 256), A=fake, B=fake, C=fake, precision=_lib.GEMM_BF16X3)
        for k, v in kw.items():
            setattr(a, k, v)
        return lib.iddgcn_rowgemm_kernel_id(ctypes.byref(a))

    assert kid() == 500
    assert kid(act=_lib.ACT_DSIGMOID, aux=fake, b_trans=1) == 501
    for R in (1, 2):
        assert kid(R=R, coef=fake, V=fake, v_idx=fake, v_rel_stride=256 * 10, v_row_stride=256,
                   act=_lib.ACT_SIGMOID) == 500 + 10 * R
    exact = lambda **kw: kid(precision=_lib.GEMM_EXACT_F32, **kw)  # noqa: E731
    assert kid(accumulate=1) == 501 and kid(accumulate=1, b_trans=1) == 501      # C += A B: old C via the aux slab
    # broadcast V (dz W_a^T), with and without the sigma' factor
    assert kid(R=2, coef=fake, V=fake, v_rel_stride=256, v_row_stride=0, act=_lib.ACT_DSIGMOID, aux=fake, b_trans=1) == 503
    assert kid(R=1, coef=fake, V=fake, v_rel_stride=256, v_row_stride=0, b_trans=1) == 502
    for kw in (dict(accumulate=1, act=_lib.ACT_SIGMOID), dict(a_idx=fake),
               dict(R=3, coef=fake, V=fake, v_rel_stride=256, v_row_stride=0, act=_lib.ACT_DSIGMOID, aux=fake),
               dict(R=2, coef=fake, coef_idx=fake, V=fake, v_idx=fake, v_rel_stride=2560, v_row_stride=256),
               dict(R=3, coef=fake, V=fake, v_idx=fake, v_rel_stride=2560, v_row_stride=256),
               dict(D=64)):
        assert kid(**kw) == exact(**kw) < 500, kw
    # the TN entry accepts the mode (invalid arguments still refused before any launch)
    assert lib.iddgcn_gemm_tn_f32(None, 32, 256, None, None, None, 1, None, 0, _lib.GEMM_BF16X3) == -3


def test_step_bytes_impl_is_a_lower_bound_of_the_measured_step():
    """engine.step_bytes_impl (round 6, bench.py step_roofline "impl"): the compulsory HBM bytes of the implemented step
    stay below the PMC-measured step they model — config 5 before the fused sigma' + TN pass (profiles/r05/cfg5/
    step_pmc_bytes_r05c5pmc.txt: read 717.6 GB + write 261.8 GB = 979 GB) — and within 10% of it; its GEMM work is
    SURVEY §8(d)'s W_gemm less the SpMMs; the fused pass saves exactly one read of do^l and x^{l-1} per layer 2-3."""
    from iddgcn_amd.engine import step_bytes_impl, step_flops
    N, R, D, M = 1_000_000, 8, 256, 40_000_000
    T = M + M // 4
    q, parts = step_bytes_impl(N, R, D, T, M, eb=2, fused_sigma_tn=False, fused_tail_head=True)
    measured = 717.6e9 + 261.8e9
    assert 0.9 * measured <= q <= measured, q / measured
    assert abs(sum(v[1] for v in parts.values()) - (step_flops(N, R, D, T, M) - 4 * M * D)) < 1e-6 * q
    qf, _ = step_bytes_impl(N, R, D, T, M, eb=2, fused_sigma_tn=True, fused_tail_head=True)
    assert q - qf == 2 * 2 * T * D * 2
