/*
 * dcfm_mex.c — MATLAB MEX gateway to libdcfm (SURVEY §8(b) callers (1), §8(f) row 1).
 * Build on a host with MATLAB:
 *     mex -R2018a dcfm_mex.c -I<repo>/include -L<pkg dir> -ldcfm
 * (not buildable in the build container: no MATLAB / mex.h there).  Commands:
 *   h = dcfm_mex('create', cfg)           cfg fields n P g K rho burnin mcmc thin as bs df ad1
 *                                         bd1 ad2 bd2 seed device inject
 *   dcfm_mex('set_data', h, Yd)           Yd n x P x g (dc:49-59 done by the caller)
 *   dcfm_mex('set_data_raw', h, Y0, cols) raw n x p0 data + int64 0-based columns (dc:48-59 on GPU)
 *   dcfm_mex('set_state', h, Lambda, ps, omega, psijh, Plam, X, Z, delta, tauh)
 *   dcfm_mex('init_state', h)             dc:68-87 on the GPU (Philox)
 *   dcfm_mex('set_draws', h, NZ, NX, NL, Gpsi, Gdelta, Gps, first, T)   injected draws
 *                                         (matlab/export_draws.m layout; cfg.inject = 1)
 *   dcfm_mex('run', h, first, count)      dc:90-197
 *   S = dcfm_mex('get_sigma', h, p)       Sigmaout (dc:194-195)
 *   e = dcfm_mex('error', h, U, s, iters) [||S-S0||_F, ||S0||_F, ||S-S0||_2] vs S0 = UU' + diag(s)
 *   dcfm_mex('set_trace', h, cap); T = dcfm_mex('get_trace', h)     chain trace (count x 4)
 *   dcfm_mex('destroy', h)
 */

#include "mex.h"
#include "dcfm.h"
#include <string.h>

static dcfm_handle *H[64];                       /* handles live across calls */

static double fld(const mxArray *s, const char *f, double dflt) {
    const mxArray *a = mxGetField(s, 0, f);
    return a ? mxGetScalar(a) : dflt;
}
static dcfm_handle *get(const mxArray *a) {
    int i = (int)mxGetScalar(a);
    if (i < 0 || i >= 64 || !H[i]) mexErrMsgIdAndTxt("dcfm:handle", "bad handle");
    return H[i];
}
static void ck(dcfm_handle *h, int rc) {
    if (rc != DCFM_OK) mexErrMsgIdAndTxt("dcfm:call", "%s", dcfm_last_error(h));
}
static void cleanup(void) { for (int i = 0; i < 64; ++i) if (H[i]) { dcfm_destroy(H[i]); H[i] = 0; } }

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
    char cmd[32];
    mexAtExit(cleanup);
    mxGetString(prhs[0], cmd, sizeof cmd);
    if (!strcmp(cmd, "create")) {
        const mxArray *s = prhs[1];
        dcfm_config c; memset(&c, 0, sizeof c);
        c.n = (int)fld(s, "n", 0);  c.P = (int)fld(s, "P", 0);  c.g = (int)fld(s, "g", 0);
        c.K = (int)fld(s, "K", 0);  c.rho = fld(s, "rho", 0);
        c.burnin = (int64_t)fld(s, "burnin", 0); c.mcmc = (int64_t)fld(s, "mcmc", 0);
        c.thin = (int64_t)fld(s, "thin", 1);
        c.as_ = fld(s, "as", 1); c.bs = fld(s, "bs", 0.3); c.df = fld(s, "df", 3);
        c.ad1 = fld(s, "ad1", 2); c.bd1 = fld(s, "bd1", 1); c.ad2 = fld(s, "ad2", 2); c.bd2 = fld(s, "bd2", 1);
        c.seed = (uint64_t)fld(s, "seed", 0); c.nranks = 1; c.device = (int)fld(s, "device", 0);
        c.flags = fld(s, "inject", 0) != 0 ? DCFM_FLAG_INJECT_DRAWS : 0u;
        int i = 0; while (i < 64 && H[i]) ++i;
        if (i == 64) mexErrMsgIdAndTxt("dcfm:handle", "too many handles");
        if (dcfm_create(&c, &H[i]) != DCFM_OK) mexErrMsgIdAndTxt("dcfm:create", "%s", dcfm_last_error(NULL));
        mexLock();
        plhs[0] = mxCreateDoubleScalar(i);
    } else if (!strcmp(cmd, "set_data")) {
        dcfm_handle *h = get(prhs[1]);
        ck(h, dcfm_set_data(h, mxGetDoubles(prhs[2])));
    } else if (!strcmp(cmd, "set_state")) {          /* Lambda ps omega psi Plam X Z delta tauh */
        dcfm_handle *h = get(prhs[1]);
        dcfm_state_view v; memset(&v, 0, sizeof v);
        v.Lambda = mxGetDoubles(prhs[2]); v.ps = mxGetDoubles(prhs[3]); v.omega = mxGetDoubles(prhs[4]);
        v.psi = mxGetDoubles(prhs[5]); v.Plam = mxGetDoubles(prhs[6]); v.X = mxGetDoubles(prhs[7]);
        v.Z = mxGetDoubles(prhs[8]); v.delta = mxGetDoubles(prhs[9]); v.tauh = mxGetDoubles(prhs[10]);
        ck(h, dcfm_set_state(h, &v));
    } else if (!strcmp(cmd, "set_data_raw")) {       /* Y0 (n x p0 double), cols (int64, 0-based) */
        dcfm_handle *h = get(prhs[1]);
        if (!mxIsInt64(prhs[3])) mexErrMsgIdAndTxt("dcfm:cols", "cols must be int64");
        ck(h, dcfm_set_data_raw(h, mxGetDoubles(prhs[2]), (int64_t)mxGetN(prhs[2]),
                                (const int64_t *)mxGetInt64s(prhs[3]), NULL, NULL));
    } else if (!strcmp(cmd, "init_state")) {
        dcfm_handle *h = get(prhs[1]);
        ck(h, dcfm_init_state(h));
    } else if (!strcmp(cmd, "set_draws")) {          /* NZ NX NL Gpsi Gdelta Gps first T */
        dcfm_handle *h = get(prhs[1]);
        dcfm_draws_view v;
        v.NZ = mxGetDoubles(prhs[2]); v.NX = mxGetDoubles(prhs[3]); v.NL = mxGetDoubles(prhs[4]);
        v.Gpsi = mxGetDoubles(prhs[5]); v.Gdelta = mxGetDoubles(prhs[6]); v.Gps = mxGetDoubles(prhs[7]);
        ck(h, dcfm_set_draws(h, &v, (int64_t)mxGetScalar(prhs[8]), (int64_t)mxGetScalar(prhs[9])));
    } else if (!strcmp(cmd, "error")) {              /* e = dcfm_mex('error', h, U, s, iters) */
        dcfm_handle *h = get(prhs[1]);
        plhs[0] = mxCreateDoubleMatrix(1, 3, mxREAL);
        ck(h, dcfm_sigma_error(h, mxGetDoubles(prhs[2]), (int32_t)mxGetN(prhs[2]), mxGetDoubles(prhs[3]),
                               (int32_t)mxGetScalar(prhs[4]), 1, mxGetDoubles(plhs[0])));
    } else if (!strcmp(cmd, "set_trace")) {
        dcfm_handle *h = get(prhs[1]);
        ck(h, dcfm_set_trace(h, (int64_t)mxGetScalar(prhs[2])));
    } else if (!strcmp(cmd, "get_trace")) {          /* count x 4, MATLAB column-major */
        dcfm_handle *h = get(prhs[1]);
        int64_t cnt = 0;
        ck(h, dcfm_get_trace(h, NULL, &cnt));
        double *rows = (double *)mxMalloc((size_t)(cnt > 0 ? cnt : 1) * 4 * sizeof(double));
        ck(h, dcfm_get_trace(h, rows, &cnt));
        plhs[0] = mxCreateDoubleMatrix((mwSize)cnt, 4, mxREAL);
        double *o = mxGetDoubles(plhs[0]);
        for (int64_t t = 0; t < cnt; ++t)
            for (int q = 0; q < 4; ++q) o[t + cnt * q] = rows[t * 4 + q];
        mxFree(rows);
    } else if (!strcmp(cmd, "run")) {
        dcfm_handle *h = get(prhs[1]);
        ck(h, dcfm_run(h, (int64_t)mxGetScalar(prhs[2]), (int64_t)mxGetScalar(prhs[3])));
    } else if (!strcmp(cmd, "get_sigma")) {          /* Sigmaout = dcfm_mex('get_sigma', h, p) */
        dcfm_handle *h = get(prhs[1]);
        mwSize p = (mwSize)mxGetScalar(prhs[2]);
        plhs[0] = mxCreateDoubleMatrix(p, p, mxREAL);
        ck(h, dcfm_get_sigma(h, mxGetDoubles(plhs[0])));
    } else if (!strcmp(cmd, "destroy")) {
        int i = (int)mxGetScalar(prhs[1]);
        if (i >= 0 && i < 64 && H[i]) { dcfm_destroy(H[i]); H[i] = 0; mexUnlock(); }
    } else {
        mexErrMsgIdAndTxt("dcfm:cmd", "unknown command %s", cmd);
    }
}
