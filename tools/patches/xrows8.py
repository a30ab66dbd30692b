"""A/B: k_xdraw with 8 rows per block (twice the blocks / CUs for the shard-message sum)."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels.hip"
s = p.read_text()
def rep(old, new, cnt=1):
    global s
    assert s.count(old) == cnt, old[:60]
    s = s.replace(old, new)
rep("""    const int i0 = blk * 16, i = i0 + c;
    const bool live = i < d.n;
    const size_t stride = (size_t)d.NP * KP;
    int nch, chunk;""", """    const int i0 = blk * XD_ROWS, i = i0 + c;
    const bool live = c < XD_ROWS && i < d.n;
    const size_t stride = (size_t)d.NP * KP;
    int nch, chunk;""")
rep("""constexpr int XD_SMEM =""", """constexpr int XD_ROWS = 8;   // rows per k_xdraw block (MFMA N = 16: lanes c >= XD_ROWS idle)
constexpr int XD_SMEM =""")
rep("""        hipLaunchKernelGGL(k_xdraw, dim3(cdiv(d.n, 16)), dim3(1024), 0, s, d, b.Sp, d.G, b.XM, b.X, dr, iter, 0,""",
    """        hipLaunchKernelGGL(k_xdraw, dim3(cdiv(d.n, XD_ROWS)), dim3(1024), 0, s, d, b.Sp, d.G, b.XM, b.X, dr, iter, 0,""")
rep("""        hipLaunchKernelGGL(k_xdraw, dim3(cdiv(d.n, 16)), dim3(1024), 0, s, d, b.xall, d.nranks, b.XM, b.X, dr,""",
    """        hipLaunchKernelGGL(k_xdraw, dim3(cdiv(d.n, XD_ROWS)), dim3(1024), 0, s, d, b.xall, d.nranks, b.XM, b.X, dr,""")
rep("""    hipLaunchKernelGGL(k_xdraw, dim3(ndel + cdiv(d.n, 16)), dim3(1024), 0, s, d, b.Sp, d.G, b.XM, b.X, dr, iter,""",
    """    hipLaunchKernelGGL(k_xdraw, dim3(ndel + cdiv(d.n, XD_ROWS)), dim3(1024), 0, s, d, b.Sp, d.G, b.XM, b.X, dr, iter,""")
rep("""        const double *p = src + (size_t)sw * chunk * stride + (size_t)i * KP + 8 * tw + 2 * q;""",
    """        const double *p = src + (size_t)sw * chunk * stride + (size_t)(c < XD_ROWS ? i : i0) * KP + 8 * tw + 2 * q;""")
p.write_text(s)
