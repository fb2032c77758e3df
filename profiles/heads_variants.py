"""Timing-only variants of the decoder heads kernel: where
does the ~16% of the launch that is not MFMA issue go?

Each variant is conv_split.hip with ONE part of the kernel removed by a text
substitution in a scratch copy of csrc/ (the committed kernel is untouched),
built as tmr_amd/libtmr_<variant>.so and selected with TMR_LIB_VARIANT by
bench.py.  Their results are WRONG by construction (no parity) -- only the
heads launch time (roofline.avg_launch_ms) and the PMC counters mean anything.

  nobar    no s_barrier at the end of each barrier step (LDS reuse races)
  nowait   no counted vmcnt wait before those barriers (DMA not awaited)
  noacc0   no initial-value (acc0) read: accumulators start at zero
  noepi    no heads epilogue: one dummy store per block
  nodma    no LDS-DMA at all (halo and weights never loaded)
  xl2band  the correlation's band staging reads 4 L2-resident rows instead of the band
  xl2a     the correlation's A fragments all come from template row 0 (L1/L2-resident)
  wsparseN / tsparseN   decoder weights' / correlation templates' hi part at
           N significant bits (WH_BITS / TH_BITS; these ARE correct builds)
  imgmajor an image's 3 units innermost in the heads grid (acc0 tile reuse; a correct build
           for 3 units per image)
  pxgN     the heads launch's XCD block groups at N pixel tiles x 32/N channel tiles (8 x 4 committed)
  xring0   the correlation's A fragments copied out of their prefetch slots (round-4 loop)
  xpf3_N / xpfwN   the correlation's A-fragment ring at N slots (3-term; < 6 / >= 6 tiles per wave)
  uprN     the upsample's output tile at N rows (32 committed; correct builds)
  gnolist / gnochain / gnorescan   the NMS greedy wave without its list test / its
           in-block chain / its overflow rescan (wrong keep lists; greedy_kernel time only)
  l2dma    every DMA re-reads the first chunk's halo / first step's weights:
           the same instruction stream with real operand data, but L2-resident
           (no MALL / HBM traffic)

    python profiles/heads_variants.py build [variants...]   # here, on the CPU
    python profiles/heads_variants.py build-rev NAME REV FILE  # FILE of csrc/ as of git REV
    python profiles/heads_variants.py clean
"""
import os
import re
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "template-matching-and-regression-mapreduce_amd")
CSRC = os.path.join(PKG, "csrc")

STEP_BARRIER = """                    wait_vmcnt(G::allowed(sg, part, HALVES));
                __builtin_amdgcn_s_barrier();"""
EPI_START = "    // ---------------- epilogue ----------------\n"


def _sub(src: str, old: str, new: str, count: int = 1) -> str:
    n = src.count(old)
    if n != count:
        raise SystemExit(f"variant substitution: expected {count} match(es), found {n}: {old[:60]!r}")
    return src.replace(old, new)


def variant_source(name: str, src: str) -> str:
    if name == "nobar":
        return _sub(src, STEP_BARRIER, "                    wait_vmcnt(G::allowed(sg, part, HALVES));\n")
    if name == "nowait":
        src = _sub(src, """                if constexpr (D == 1)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else
                    wait_vmcnt(G::allowed(sg, part, HALVES));""", "")
        return src
    if name == "noacc0":
        return _sub(src, "    if (a.acc_init && (a.flags & TMR_SPLIT_TILED_INIT) && (a.flags & TMR_SPLIT_INIT_BF16)) {",
                    "    if (false) {")
    if name == "noepi":
        return _sub(src, EPI_START, EPI_START + """    if constexpr (EPI == 1) {
        float s_ = 0.0f;
#pragma unroll
        for (int in = 0; in < NIN; ++in)
#pragma unroll
            for (int jp = 0; jp < 8; ++jp) s_ += acc[in][jp][0];
        if (s_ == 1234.5f) a.partials[tid] = s_;  // keeps the main loop alive
        return;
    }
""")
    if name == "nodma":
        return _sub(src, "    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);",
                    "    (void)r; (void)dst; (void)voff; (void)soff;")
    if name.startswith("wsparse"):  # weights' hi part to N significant bits (wsparse8, wsparse11)
        return re.sub(r"constexpr int WH_BITS = \d+;", f"constexpr int WH_BITS = {int(name[7:])};", src, count=1)
    if name == "xl2band":  # correlation band staging reads 4 L2-resident rows (timing only)
        return _sub(src, "if (e < n4 && yy >= 0 && yy < H) v[k] = reinterpret_cast<const float4 *>(fc + (size_t)yy * W)[cc];",
                    "if (e < n4 && yy >= 0 && yy < H) v[k] = reinterpret_cast<const float4 *>(a.f + (size_t)(yy & 3) * W)[cc];")
    if name == "xl2a":  # correlation A fragments all read from template row 0 (L1/L2-resident; timing only)
        return _sub(src, "return *reinterpret_cast<const V *>(arow + (size_t)((i * NK + nk) * 2 + term) * AFRAG);",
                    "return *reinterpret_cast<const V *>(arow + (size_t)((0 * i + nk) * 2 + term) * AFRAG);")
    if name.startswith("tsparse"):  # correlation templates' hi part (xcorr.hip TH_BITS)
        return _sub(src, "constexpr int TH_BITS = 11;", f"constexpr int TH_BITS = {int(name[7:])};")
    if name == "l2dma":
        src = _sub(src, "        const uint32_t soff = (uint32_t)(s0 ? hc : hc - h0) * cstride;",
                   "        const uint32_t soff = 0u * (uint32_t)(s0 ? hc : hc - h0) * cstride;")
        src = _sub(src, "buffer_lds16(wr, (lds_ptr_t)w_dst(g, ipt, m), wlane, w_src(g, ipt, m));",
                   "buffer_lds16(wr, (lds_ptr_t)w_dst(g, ipt, m), wlane, w_src(0, ipt, m));")
        src = _sub(src, "const uint32_t src = (uint32_t)(sgx * G::tps(px) + tl) * tapstride + (uint32_t)cx * a.Npad * WREC + wnt +",
                   "const uint32_t src = (uint32_t)tl * tapstride + wnt +")
        return src
    if name == "imgmajor":  # an image's E = 3 units innermost in the block order
        # (correct results for U % 3 == 0 with 3 units per image, e.g. config B): the 3 blocks of an
        # image at one (pixel tile, channel tile) are consecutive on one XCD, so its acc0 tile is
        # fetched from HBM once and served from L2 to the other two
        # Only the heads launch (EPI == 1) with a unit count divisible by 3 is remapped: the store,
        # projection and bias-plane launches (U = images, or 1) keep the unit-major order (round 5's
        # first build remapped every launch and faulted on the bias plane's U = 1: u out of range)
        return _sub(src, """        const int per_unit = a.NT * a.MT;
        u = L / per_unit;
        const int r = L - u * per_unit;""", """        const int per_unit = a.NT * a.MT;
        int r;
        if (EPI == 1 && a.U % 3 == 0) {
            const int ub = L / (3 * per_unit), rr = L - ub * 3 * per_unit;
            u = ub * 3 + rr % 3;
            r = rr / 3;
        } else {
            u = L / per_unit;
            r = L - u * per_unit;
        }""")
    if name.startswith("pxg"):  # heads XCD block groups: PXG pixel tiles x (32 / PXG) channel tiles
        pxg = int(name[3:])
        return _sub(src, "constexpr int PXG = 8, NG = 4;", f"constexpr int PXG = {pxg}, NG = {32 // pxg};")
    if name == "xring0":  # the correlation's A fragments copied out of the prefetch slots (round 4 form)
        return _sub(src, "constexpr int XCORR_RING = 1;", "constexpr int XCORR_RING = 0;")
    if name.startswith("xpf3_"):  # ring slots of the 3-term kernel below 6 tiles per wave
        return _sub(src, "constexpr int XRING_PF1 = 4, XRING_PF3 = 2,", f"constexpr int XRING_PF1 = 4, XRING_PF3 = {int(name[5:])},")
    if name.startswith("xpfw"):  # ring slots of the 3-term kernel at >= 6 tiles per wave
        return _sub(src, "XRING_PF3_WIDE = 3;", f"XRING_PF3_WIDE = {int(name[4:])};")
    if name.startswith("upr"):  # upsample2x output tile rows (upr64, upr128)
        return _sub(src, "constexpr int UPT_R = 32, UPT_C = 128;", f"constexpr int UPT_R = {int(name[3:])}, UPT_C = 128;")
    if name == "gnolist":
        return _sub(src, "        bool rem = rem32 != 0;", "        bool rem = false; (void)rem32;")
    if name == "gnochain":
        return _sub(src, "        for (uint64_t avail = ~word; avail;) {  // the surviving rows, lowest first",
                    "        kept = ~word; (void)dlo; (void)dhi;\n        for (uint64_t avail = 0; avail;) {")
    if name == "gnorescan":
        return _sub(src, "        for (uint64_t ovf = __ballot(i < n && lc > CAP && !rem); ovf; ovf &= ovf - 1) {",
                    "        for (uint64_t ovf = 0; ovf; ovf &= ovf - 1) {")
    raise SystemExit(f"unknown variant {name}")


def variant_file(name: str) -> str:
    if name.startswith("g"):
        return "nms.hip"
    if name.startswith("upr"):
        return "upsample_heads.hip"
    return "xcorr.hip" if name.startswith(("tsparse", "xl2band", "xl2a", "xring", "xpf")) else "conv_split.hip"


VARIANTS = ["nobar", "nowait", "noacc0", "noepi", "nodma", "l2dma"]


def build(names, rev_file=None):
    for name in names:
        scratch = os.path.join(PKG, f"build_var_{name}")
        src_dir = os.path.join(scratch, "csrc")
        shutil.rmtree(scratch, ignore_errors=True)
        shutil.copytree(CSRC, src_dir)
        # the scratch csrc sits one level deeper: point its include path at the repo
        for f in os.listdir(src_dir):
            if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile":
                p = os.path.join(src_dir, f)
                txt = open(p).read().replace("../../include/", "../../../include/")
                if rev_file is not None and f == rev_file[1]:
                    rel = os.path.relpath(os.path.join(CSRC, f), REPO)
                    txt = subprocess.run(["git", "-C", REPO, "show", f"{rev_file[0]}:{rel}"], check=True,
                                         capture_output=True, text=True).stdout
                    txt = txt.replace("../../include/", "../../../include/")
                elif rev_file is None and f == variant_file(name):
                    txt = variant_source(name, txt)
                with open(p, "w") as fh:
                    fh.write(txt)
        out = os.path.join(PKG, f"libtmr_{name}.so")
        subprocess.check_call(["make", "-s", "-j8", "-C", src_dir, f"OUT={out}", f"OBJDIR={scratch}/obj"])
        shutil.rmtree(scratch, ignore_errors=True)
        print("built", out)


def clean():
    for f in os.listdir(PKG):
        if f.startswith("libtmr_") and f.endswith(".so"):
            os.remove(os.path.join(PKG, f))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "clean":
        clean()
    elif len(sys.argv) > 1 and sys.argv[1] == "build-rev":
        build([sys.argv[2]], (sys.argv[3], sys.argv[4]))
    else:
        build(sys.argv[2:] or VARIANTS)
