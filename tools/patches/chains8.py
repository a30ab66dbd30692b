"""A/B: 8 independent MFMA accumulator chains per wave in the Y passes (k_cpass, the W tiles
of k_wcol / k_wpass): alternate k-steps go to a second accumulator set, summed at the end."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels.hip"
s = p.read_text()
def rep(old, new):
    global s
    assert s.count(old) == 1, old[:60]
    s = s.replace(old, new)
# ---- wpass_tile
rep("""    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int nch = d.PP >> 3;""", """    d4 acc[2][2], acc2[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = acc2[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    const int nch = d.PP >> 3;""")
rep("""        acc[0][0] = mfma16x16x4(y0.y, b10, acc[0][0]);                              \\
        acc[0][1] = mfma16x16x4(y0.y, b11, acc[0][1]);                              \\
        acc[1][0] = mfma16x16x4(y1.y, b10, acc[1][0]);                              \\
        acc[1][1] = mfma16x16x4(y1.y, b11, acc[1][1]);                              \\""",
"""        acc2[0][0] = mfma16x16x4(y0.y, b10, acc2[0][0]);                            \\
        acc2[0][1] = mfma16x16x4(y0.y, b11, acc2[0][1]);                            \\
        acc2[1][0] = mfma16x16x4(y1.y, b10, acc2[1][0]);                            \\
        acc2[1][1] = mfma16x16x4(y1.y, b11, acc2[1][1]);                            \\""")
rep("""#undef WP_LOAD
#undef WP_MMA
    // D row = q + 4g (row i), col = r (k = 2r + tb)""", """#undef WP_LOAD
#undef WP_MMA
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] += acc2[a][b];
    // D row = q + 4g (row i), col = r (k = 2r + tb)""")
# ---- cpass_wave: acc2 set for odd u
rep("""                                           const double *__restrict__ Za, int s0, int nsw,
                                           int q, d4 (&acc)[2][2]) {""", """                                           const double *__restrict__ Za, int s0, int nsw,
                                           int q, d4 (&acc)[2][2], d4 (&acc2)[2][2]) {""")
rep("""            const double a0 = (IS_E && SAME_T) ? e0 : y[u].x, a1 = (IS_E && SAME_T) ? e1 : y[u].y;
            acc[0][0] = mfma16x16x4(a0, e0, acc[0][0]);
            acc[0][1] = mfma16x16x4(a0, e1, acc[0][1]);
            acc[1][0] = mfma16x16x4(a1, e0, acc[1][0]);
            acc[1][1] = mfma16x16x4(a1, e1, acc[1][1]);""", """            const double a0 = (IS_E && SAME_T) ? e0 : y[u].x, a1 = (IS_E && SAME_T) ? e1 : y[u].y;
            d4 (&ac)[2][2] = (u & 1) ? acc2 : acc;
            ac[0][0] = mfma16x16x4(a0, e0, ac[0][0]);
            ac[0][1] = mfma16x16x4(a0, e1, ac[0][1]);
            ac[1][0] = mfma16x16x4(a1, e0, ac[1][0]);
            ac[1][1] = mfma16x16x4(a1, e1, ac[1][1]);""")
rep("""    d4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    if (!isE) cpass_wave<KW, false, false>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc);
    else if (te == kt) cpass_wave<KW, true, true>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc);
    else cpass_wave<KW, true, false>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc);""", """    d4 acc[2][2], acc2[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = acc2[a][b] = d4{0.0, 0.0, 0.0, 0.0};
    if (!isE) cpass_wave<KW, false, false>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc, acc2);
    else if (te == kt) cpass_wave<KW, true, true>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc, acc2);
    else cpass_wave<KW, true, false>(d, Yp, Xp, Zp, Xa, Za, wave * nsw, nsw, q, acc, acc2);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] += acc2[a][b];""")
p.write_text(s)
