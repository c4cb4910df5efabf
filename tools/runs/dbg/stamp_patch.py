"""Instrumented copy of iddgcn_hip.hip for per-phase timing of rowgemm256_b3_kernel's main loop (round 6).

Writes <out>/iddgcn_amd/csrc/iddgcn_hip.hip (+ include/) with s_memtime stamps at five points of each of the first
16 tiles of workgroups 0..15, waves 0 (early half of a SIMD) and 4 (late half of the same SIMD):
  0 loop top (after the previous barrier)   1 before the MFMA phase   2 after it (the accumulators complete)
  3 before the barrier (post-MFMA work done) 4 after the barrier
plus s_memrealtime (100 MHz) beside stamps 0 and 4, and an exported iddgcn_dbg_stamps(dst, bytes) that copies the
table to the host.  Vector stores from lane 0 only.  Not product code: tools/runs/dbg/stamp_fwd.py drives it.

usage: python tools/runs/dbg/stamp_patch.py OUTDIR [rowgemm|rowgemm_fine|sigma_tn]
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rep(src, old, new, count=1):
    n = src.count(old)
    if n != count:
        raise SystemExit(f"pattern found {n} times, expected {count}: {old[:80]!r}")
    return src.replace(old, new)


def patch_sigma_tn(src):
    """Stamps in sigma_tn_b3_kernel's loop: 0 top, 1 after staging, 2 after the sigma' MFMAs (acc complete), 3 after the
    epilogue, 4 after the TN MFMAs (issued), 5 after the conversions, 6 after the barrier; 7 = s_memrealtime at 0."""
    src = rep(src, "            const bool stager = ROLES == 0 || wave < 4;\n",
              "            const bool stager = ROLES == 0 || wave < 4;\n"
              "            const bool stamp_on = bx < 16 && (wave == 0 || wave == 4);\n"
              "            const int sidx = bx * 2 + (wave >= 4 ? 1 : 0);\n"
              "#define STAMP(k) do { if (stamp_on && (t - t_beg) < 16) { const unsigned long long ts_ = "
              "__builtin_amdgcn_s_memtime(); if (lane == 0) g_stamp[(sidx * 16 + (int)(t - t_beg)) * 8 + (k)] = ts_; } } "
              "while (0)\n")
    src = rep(src, "                const bool more = t + 1 < t_end;\n                if (more && stager) {\n",
              "                const bool more = t + 1 < t_end; STAMP(0);\n"
              "                if (stamp_on && (t - t_beg) < 16 && lane == 0) g_stamp[(sidx * 16 + (int)(t - t_beg)) * 8 + 7] = "
              "__builtin_amdgcn_s_memrealtime();\n"
              "                if (more && stager) {\n")
    src = rep(src, "                f32x4 acc[2];\n                mfma_sigma(b, acc);\n"
                   "                const int ns = epilogue(t, b, acc);\n",
              "                STAMP(1); f32x4 acc[2];\n                mfma_sigma(b, acc);\n"
              "                asm volatile(\"\" :: \"v\"(acc[0]), \"v\"(acc[1]) : \"memory\"); STAMP(2);\n"
              "                const int ns = epilogue(t, b, acc); STAMP(3);\n")
    src = rep(src, "                mfma_tn(b);\n                if (ROLES != 2",
              "                mfma_tn(b); STAMP(4);\n                if (ROLES != 2")
    src = rep(src, "                asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");\n"
                   "                __builtin_amdgcn_s_barrier();\n                asm volatile(\"\" ::: \"memory\");\n"
                   "                b ^= 1;\n",
              "                asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\"); STAMP(5);\n"
              "                __builtin_amdgcn_s_barrier(); STAMP(6);\n                asm volatile(\"\" ::: \"memory\");\n"
              "                b ^= 1;\n")
    return src


FINE_LOOP = r"""        f32x4 acc[2];                                                                                \
        int b = 0;                                                                                   \
        for (long long t = t_beg; t < t_end; ++t) {                                                  \
            const bool more = t + 1 < t_end; STAMPF(0);                                              \
            const int nA = dma_A(t + 1, b ^ 1); STAMPF(1);                                           \
            int after_A = 0;                                                                         \
            if (LATE && t > t_beg) {                                                                 \
                wait_vm(nA + 4); STAMPX(0); wait_vm(nA + 1); STAMPX(1); wait_vm(nA); STAMPF(2);                                                              \
                after_A += epilogue(t - 1, acc); STAMPF(3);                                          \
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                   \
                after_A += dma_slabs(t); STAMPF(4);                                                  \
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                   \
                after_A += dma_idx(t + 1); STAMPF(5);                                                \
            }                                                                                        \
            STAMPF(6); mfma_tile(b, acc); asm volatile("" :: "v"(acc[0]), "v"(acc[1]) : "memory"); STAMPF(7); \
            if (LATE) {                                                                              \
                if (more) {                                                                          \
                    wait_vm(after_A); STAMPF(8);                                                     \
                    convert(b ^ 1); STAMPF(9);                                                       \
                }                                                                                    \
            } else {                                                                                 \
                wait_vm(nA + 4); STAMPX(2); wait_vm(nA + 1); STAMPX(3); wait_vm(nA); STAMPF(8);                                                              \
                after_A += epilogue(t, acc); STAMPF(9);                                              \
                if (more) {                                                                          \
                    wait_vm(after_A); STAMPF(10);                                                    \
                    convert(b ^ 1); STAMPF(11);                                                      \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                               \
                    dma_slabs(t + 1); STAMPF(12);                                                    \
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                               \
                    dma_idx(t + 2); STAMPF(13);                                                      \
                }                                                                                    \
            }                                                                                        \
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); STAMPF(14);                           \
            __builtin_amdgcn_s_barrier();                                                            \
            asm volatile("" ::: "memory"); STAMPF(15);                                               \
            b ^= 1;                                                                                  \
        }                                                                                            \
"""


def patch_rowgemm_fine(src):
    """16 stamps per tile in rowgemm256_b3_kernel's loop (see FINE_LOOP); table [32][16][16]."""
    i0 = src.index("#define B3_MAIN_LOOP(LATE)")
    i1 = src.index("        if (LATE) {                                                                                  \\\n"
                   "            asm volatile(\"s_waitcnt vmcnt(0)\"", i0)
    head = src[i0:src.index("\n", i0) + 1] + "    {                                                                                                \\\n"
    src = src[:i0] + ("    const bool stamp_on = bx < 16 && (wave == 0 || wave == 4);\n"
                      "    const int sidx = bx * 2 + (wave >= 4 ? 1 : 0);\n"
                      "#define STAMPF(k) do { if (stamp_on && (t - t_beg) < 16) { const unsigned long long ts_ = "
                      "__builtin_amdgcn_s_memtime(); if (lane == 0) g_stampf[(sidx * 16 + (int)(t - t_beg)) * 16 + (k)] = ts_; } } "
                      "while (0)\n"
                      "#define STAMPX(k) do { if (stamp_on && (t - t_beg) < 16) { const unsigned long long ts_ = "
                      "__builtin_amdgcn_s_memtime(); if (lane == 0) g_stampx[(sidx * 16 + (int)(t - t_beg)) * 4 + (k)] = ts_; } } "
                      "while (0)\n") + head + FINE_LOOP + src[i1:]
    return src


def main(out, kernel="rowgemm"):
    os.makedirs(os.path.join(out, "iddgcn_amd", "csrc"), exist_ok=True)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(out, "include"), dirs_exist_ok=True)
    src = open(os.path.join(ROOT, "iddgcn_amd", "csrc", "iddgcn_hip.hip")).read()
    src = rep(src, "}  // namespace rb3\n",
              "}  // namespace rb3\n"
              "__device__ unsigned long long g_stamp[32 * 16 * 8];\n")
    if kernel == "rowgemm_fine":
        src = rep(src, "__device__ unsigned long long g_stamp[32 * 16 * 8];\n",
                  "__device__ unsigned long long g_stamp[32 * 16 * 8];\n__device__ unsigned long long g_stampf[32 * 16 * 16];\n"
                  "__device__ unsigned long long g_stampx[32 * 16 * 4];\n")
        src = patch_rowgemm_fine(src)
        src += ('\nextern "C" int iddgcn_dbg_stamps(void* dst, long long bytes) {\n'
                '    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stampf), (size_t)bytes, 0, hipMemcpyDeviceToHost);\n'
                '}\n'
                'extern "C" int iddgcn_dbg_stampx(void* dst, long long bytes) {\n'
                '    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stampx), (size_t)bytes, 0, hipMemcpyDeviceToHost);\n'
                '}\n')
        open(os.path.join(out, "iddgcn_amd", "csrc", "iddgcn_hip.hip"), "w").write(src)
        return
    if kernel == "sigma_tn":
        src = patch_sigma_tn(src)
        src += ('\nextern "C" int iddgcn_dbg_stamps(void* dst, long long bytes) {\n'
                '    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamp), (size_t)bytes, 0, hipMemcpyDeviceToHost);\n'
                '}\n')
        open(os.path.join(out, "iddgcn_amd", "csrc", "iddgcn_hip.hip"), "w").write(src)
        return
    # stamp state, before the loop macro
    src = rep(src, "#define B3_MAIN_LOOP(LATE)",
              "    const bool stamp_on = bx < 16 && (wave == 0 || wave == 4);\n"
              "    const int sidx = bx * 2 + (wave >= 4 ? 1 : 0);\n"
              "#define STAMP(k) do { if (stamp_on && (t - t_beg) < 16) { const unsigned long long ts_ = "
              "__builtin_amdgcn_s_memtime(); if (lane == 0) g_stamp[(sidx * 16 + (int)(t - t_beg)) * 8 + (k)] = ts_; } } "
              "while (0)\n"
              "#define STAMPR(k) do { if (stamp_on && (t - t_beg) < 16) { const unsigned long long ts_ = "
              "__builtin_amdgcn_s_memrealtime(); if (lane == 0) g_stamp[(sidx * 16 + (int)(t - t_beg)) * 8 + (k)] = ts_; } } "
              "while (0)\n"
              "#define B3_MAIN_LOOP(LATE)")
    src = rep(src, "            const bool more = t + 1 < t_end;                                                         \\",
              "            const bool more = t + 1 < t_end; STAMP(0); STAMPR(5);                                    \\")
    src = rep(src, "            mfma_tile(b, acc);                                                                       \\",
              "            STAMP(1); mfma_tile(b, acc); asm volatile(\"\" :: \"v\"(acc[0]), \"v\"(acc[1]) : \"memory\"); "
              "STAMP(2); \\")
    src = rep(src, "            asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");                                       \\\n"
                   "            __builtin_amdgcn_s_barrier();                                                            \\\n"
                   "            asm volatile(\"\" ::: \"memory\");                                                           \\\n"
                   "            b ^= 1;                                                                                  \\",
              "            asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");                                       \\\n"
              "            STAMP(3);                                                                                \\\n"
              "            __builtin_amdgcn_s_barrier();                                                            \\\n"
              "            asm volatile(\"\" ::: \"memory\");                                                           \\\n"
              "            STAMP(4); STAMPR(6);                                                                     \\\n"
              "            b ^= 1;                                                                                  \\")
    src += ('\nextern "C" int iddgcn_dbg_stamps(void* dst, long long bytes) {\n'
            '    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamp), (size_t)bytes, 0, hipMemcpyDeviceToHost);\n'
            '}\n')
    open(os.path.join(out, "iddgcn_amd", "csrc", "iddgcn_hip.hip"), "w").write(src)


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))
