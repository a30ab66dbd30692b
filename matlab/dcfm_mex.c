/*
 * dcfm_mex.c — MATLAB MEX gateway to libdcfm (SURVEY §8(b) callers (1), §8(f) row 1).
 * Build on a host with MATLAB:
 *     mex -R2018a dcfm_mex.c -I<repo>/include -L<pkg dir> -ldcfm
 * (the build container has no MATLAB; tests/test_mex_gateway.py compiles this file against
 * a mock of the mx / mex API and drives it, argument checking on the CPU and a whole chain
 * on the GPU).  Commands:
 *   h = dcfm_mex('create', cfg)           cfg fields n P g K rho burnin mcmc thin as bs df ad1
 *                                         bd1 ad2 bd2 seed device inject asm_batch
 *   dcfm_mex('set_data', h, Yd)           Yd n x P x g (dc:49-59 done by the caller)
 *   dcfm_mex('set_data_raw', h, Y0, cols) raw n x p0 data + int64 0-based columns (dc:48-59 on GPU)
 *   dcfm_mex('set_state', h, Lambda, ps, omega, psijh, Plam, X, Z, delta, tauh)
 *   dcfm_mex('init_state', h)             dc:68-87 on the GPU (Philox)
 *   dcfm_mex('set_draws', h, NZ, NX, NL, Gpsi, Gdelta, Gps, first, T)   injected draws
 *                                         (matlab/export_draws.m layout; cfg.inject = 1)
 *   dcfm_mex('run', h, first, count)      dc:90-197
 *   [Lambda, ps, omega, psijh, Plam, X, Z, eta, delta, tauh] = dcfm_mex('get_state', h)
 *   S = dcfm_mex('get_sigma', h)          Sigmaout (dc:194-195), p x p from the handle
 *   e = dcfm_mex('error', h, U, s, iters) [||S-S0||_F, ||S0||_F, ||S-S0||_2] vs S0 = UU' + diag(s)
 *   dcfm_mex('set_trace', h, cap); T = dcfm_mex('get_trace', h)     chain trace (count x 4)
 *   dcfm_mex('destroy', h)
 * Every array argument is checked (class double, real, element count from the handle's
 * own dimensions) before the library sees its pointer: the library reads and writes at
 * config-derived sizes, so a wrong-sized MATLAB array must never reach it.
 */

#include "mex.h"
#include "dcfm.h"
#include <stdint.h>
#include <string.h>

#define NSLOT 64
typedef struct {
    dcfm_handle *h;
    int64_t n, P, g, K;        /* this handle's dimensions (single rank: g_local = g) */
} slot;
static slot S[NSLOT];          /* handles live across calls */

static void cleanup(void) {
    for (int i = 0; i < NSLOT; ++i)
        if (S[i].h) { dcfm_destroy(S[i].h); S[i].h = 0; }
}

static double fld(const mxArray *s, const char *f, double dflt) {
    const mxArray *a = mxGetField(s, 0, f);
    if (!a) return dflt;
    if (!mxIsDouble(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != 1)
        mexErrMsgIdAndTxt("dcfm:cfg", "cfg.%s must be a real double scalar", f);
    return mxGetScalar(a);
}
static double scalar(const mxArray *a, const char *what) {
    if (!mxIsDouble(a) || mxIsComplex(a) || mxGetNumberOfElements(a) != 1)
        mexErrMsgIdAndTxt("dcfm:arg", "%s must be a real double scalar", what);
    return mxGetScalar(a);
}
static slot *get(const mxArray *a) {
    const double v = scalar(a, "handle");
    const int i = (int)v;
    if ((double)i != v || i < 0 || i >= NSLOT || !S[i].h) mexErrMsgIdAndTxt("dcfm:handle", "bad handle");
    return &S[i];
}
/* a real double array of exactly `numel` elements; its data pointer */
static double *need(const mxArray *a, int64_t numel, const char *what) {
    if (!mxIsDouble(a) || mxIsComplex(a))
        mexErrMsgIdAndTxt("dcfm:arg", "%s must be a real double array", what);
    if ((int64_t)mxGetNumberOfElements(a) != numel)
        mexErrMsgIdAndTxt("dcfm:arg", "%s must have %lld elements, got %lld", what, (long long)numel,
                          (long long)mxGetNumberOfElements(a));
    return mxGetDoubles(a);
}
static void nargs(int nrhs, int want, const char *cmd) {
    if (nrhs != want) mexErrMsgIdAndTxt("dcfm:nargs", "'%s' takes %d arguments, got %d", cmd, want - 1, nrhs - 1);
}
static void ck(dcfm_handle *h, int rc) {
    if (rc != DCFM_OK) mexErrMsgIdAndTxt("dcfm:call", "%s", dcfm_last_error(h));
}

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
    char cmd[32];
    mexAtExit(cleanup);
    if (nrhs < 1 || !mxIsChar(prhs[0]) || mxGetString(prhs[0], cmd, sizeof cmd) != 0)
        mexErrMsgIdAndTxt("dcfm:cmd", "first argument must be a command string");
    if (!strcmp(cmd, "create")) {
        nargs(nrhs, 2, cmd);
        const mxArray *s = prhs[1];
        if (!mxIsStruct(s)) mexErrMsgIdAndTxt("dcfm:cfg", "cfg must be a struct");
        dcfm_config c;
        memset(&c, 0, sizeof c);
        c.n = (int32_t)fld(s, "n", 0);  c.P = (int32_t)fld(s, "P", 0);  c.g = (int32_t)fld(s, "g", 0);
        c.K = (int32_t)fld(s, "K", 0);  c.rho = fld(s, "rho", 0);
        c.burnin = (int64_t)fld(s, "burnin", 0); c.mcmc = (int64_t)fld(s, "mcmc", 0);
        c.thin = (int64_t)fld(s, "thin", 1);
        c.as_ = fld(s, "as", 1); c.bs = fld(s, "bs", 0.3); c.df = fld(s, "df", 3);
        c.ad1 = fld(s, "ad1", 2); c.bd1 = fld(s, "bd1", 1); c.ad2 = fld(s, "ad2", 2); c.bd2 = fld(s, "bd2", 1);
        c.seed = (uint64_t)fld(s, "seed", 0); c.nranks = 1; c.device = (int32_t)fld(s, "device", 0);
        c.flags = fld(s, "inject", 0) != 0 ? DCFM_FLAG_INJECT_DRAWS : 0u;
        c.asm_batch = (int32_t)fld(s, "asm_batch", 0);
        int i = 0;
        while (i < NSLOT && S[i].h) ++i;
        if (i == NSLOT) mexErrMsgIdAndTxt("dcfm:handle", "too many handles");
        if (dcfm_create(&c, &S[i].h) != DCFM_OK) {
            S[i].h = 0;
            mexErrMsgIdAndTxt("dcfm:create", "%s", dcfm_last_error(NULL));
        }
        S[i].n = c.n; S[i].P = c.P; S[i].g = c.g; S[i].K = c.K;
        mexLock();
        plhs[0] = mxCreateDoubleScalar(i);
    } else if (!strcmp(cmd, "set_data")) {
        nargs(nrhs, 3, cmd);
        slot *t = get(prhs[1]);
        ck(t->h, dcfm_set_data(t->h, need(prhs[2], t->n * t->P * t->g, "Yd (n x P x g)")));
    } else if (!strcmp(cmd, "set_state")) {          /* Lambda ps omega psi Plam X Z delta tauh */
        nargs(nrhs, 11, cmd);
        slot *t = get(prhs[1]);
        const int64_t PKg = t->P * t->K * t->g, Pg = t->P * t->g, nK = t->n * t->K, Kg = t->K * t->g;
        dcfm_state_view v;
        memset(&v, 0, sizeof v);
        v.Lambda = need(prhs[2], PKg, "Lambda (P x K x g)");
        v.ps = need(prhs[3], Pg, "ps (P x 1 x g)");
        v.omega = need(prhs[4], Pg, "omega (P x g)");
        v.psi = need(prhs[5], PKg, "psijh (P x K x g)");
        v.Plam = need(prhs[6], PKg, "Plam (P x K x g)");
        v.X = need(prhs[7], nK, "X (n x K)");
        v.Z = need(prhs[8], nK * t->g, "Z (n x K x g)");
        v.delta = need(prhs[9], Kg, "delta (K x 1 x g)");
        v.tauh = need(prhs[10], Kg, "tauh (K x 1 x g)");
        ck(t->h, dcfm_set_state(t->h, &v));
    } else if (!strcmp(cmd, "get_state")) {
        nargs(nrhs, 2, cmd);
        slot *t = get(prhs[1]);
        const mwSize P = (mwSize)t->P, K = (mwSize)t->K, g = (mwSize)t->g, n = (mwSize)t->n;
        const mwSize dPKg[3] = {P, K, g}, dP1g[3] = {P, 1, g}, dnKg[3] = {n, K, g}, dK1g[3] = {K, 1, g};
        mxArray *o[10];
        o[0] = mxCreateNumericArray(3, dPKg, mxDOUBLE_CLASS, mxREAL);   /* Lambda */
        o[1] = mxCreateNumericArray(3, dP1g, mxDOUBLE_CLASS, mxREAL);   /* ps */
        o[2] = mxCreateDoubleMatrix(P, g, mxREAL);                      /* omega */
        o[3] = mxCreateNumericArray(3, dPKg, mxDOUBLE_CLASS, mxREAL);   /* psijh */
        o[4] = mxCreateNumericArray(3, dPKg, mxDOUBLE_CLASS, mxREAL);   /* Plam */
        o[5] = mxCreateDoubleMatrix(n, K, mxREAL);                      /* X */
        o[6] = mxCreateNumericArray(3, dnKg, mxDOUBLE_CLASS, mxREAL);   /* Z */
        o[7] = mxCreateNumericArray(3, dnKg, mxDOUBLE_CLASS, mxREAL);   /* eta */
        o[8] = mxCreateNumericArray(3, dK1g, mxDOUBLE_CLASS, mxREAL);   /* delta */
        o[9] = mxCreateNumericArray(3, dK1g, mxDOUBLE_CLASS, mxREAL);   /* tauh */
        dcfm_state_view v;
        v.Lambda = mxGetDoubles(o[0]); v.ps = mxGetDoubles(o[1]); v.omega = mxGetDoubles(o[2]);
        v.psi = mxGetDoubles(o[3]); v.Plam = mxGetDoubles(o[4]); v.X = mxGetDoubles(o[5]);
        v.Z = mxGetDoubles(o[6]); v.eta = mxGetDoubles(o[7]); v.delta = mxGetDoubles(o[8]);
        v.tauh = mxGetDoubles(o[9]);
        ck(t->h, dcfm_get_state(t->h, &v));
        for (int q = 0; q < 10; ++q) {
            if (q < (nlhs < 1 ? 1 : nlhs)) plhs[q] = o[q];
            else mxDestroyArray(o[q]);
        }
    } else if (!strcmp(cmd, "set_data_raw")) {       /* Y0 (n x p0 double), cols (int64, 0-based) */
        nargs(nrhs, 4, cmd);
        slot *t = get(prhs[1]);
        const mxArray *Y = prhs[2], *cols = prhs[3];
        if (!mxIsDouble(Y) || mxIsComplex(Y) || (int64_t)mxGetM(Y) != t->n)
            mexErrMsgIdAndTxt("dcfm:arg", "Y0 must be a real double n x p0 matrix (n = %lld)", (long long)t->n);
        const int64_t p0 = (int64_t)mxGetN(Y);
        if (!mxIsInt64(cols) || (int64_t)mxGetNumberOfElements(cols) != t->P * t->g)
            mexErrMsgIdAndTxt("dcfm:cols", "cols must be int64 with P*g = %lld elements", (long long)(t->P * t->g));
        const int64_t *cv = (const int64_t *)mxGetInt64s(cols);
        for (int64_t e = 0; e < t->P * t->g; ++e)
            if (cv[e] < 0 || cv[e] >= p0) mexErrMsgIdAndTxt("dcfm:cols", "cols(%lld) = %lld outside 0..p0-1",
                                                             (long long)(e + 1), (long long)cv[e]);
        ck(t->h, dcfm_set_data_raw(t->h, mxGetDoubles(Y), p0, cv, NULL, NULL));
    } else if (!strcmp(cmd, "init_state")) {
        nargs(nrhs, 2, cmd);
        slot *t = get(prhs[1]);
        ck(t->h, dcfm_init_state(t->h));
    } else if (!strcmp(cmd, "set_draws")) {          /* NZ NX NL Gpsi Gdelta Gps first T */
        nargs(nrhs, 10, cmd);
        slot *t = get(prhs[1]);
        const double first = scalar(prhs[8], "first"), T = scalar(prhs[9], "T");
        if (T < 1 || T != (double)(int64_t)T || first != (double)(int64_t)first)
            mexErrMsgIdAndTxt("dcfm:arg", "first and T must be integers, T >= 1");
        const int64_t nT = (int64_t)T;
        dcfm_draws_view v;
        v.NZ = need(prhs[2], t->K * t->n * t->g * nT, "NZ (K x n x g x T)");
        v.NX = need(prhs[3], t->K * t->n * nT, "NX (K x n x T)");
        v.NL = need(prhs[4], t->K * t->P * t->g * nT, "NL (K x P x g x T)");
        v.Gpsi = need(prhs[5], t->P * t->K * t->g * nT, "Gpsi (P x K x g x T)");
        v.Gdelta = need(prhs[6], t->K * t->g * nT, "Gdelta (K x g x T)");
        v.Gps = need(prhs[7], t->P * t->g * nT, "Gps (P x g x T)");
        ck(t->h, dcfm_set_draws(t->h, &v, (int64_t)first, nT));
    } else if (!strcmp(cmd, "error")) {              /* e = dcfm_mex('error', h, U, s, iters) */
        nargs(nrhs, 5, cmd);
        slot *t = get(prhs[1]);
        const int64_t p = t->P * t->g;
        const mxArray *U = prhs[2];
        if (!mxIsDouble(U) || mxIsComplex(U) || (int64_t)mxGetM(U) != p || mxGetN(U) < 1 || mxGetN(U) > 32)
            mexErrMsgIdAndTxt("dcfm:arg", "U must be a real double p x r matrix, p = %lld, 1 <= r <= 32", (long long)p);
        const double *sv = need(prhs[3], p, "s (p x 1)");
        const double it = scalar(prhs[4], "iters");
        if (it < 0 || it != (double)(int32_t)it) mexErrMsgIdAndTxt("dcfm:arg", "iters must be a non-negative integer");
        plhs[0] = mxCreateDoubleMatrix(1, 3, mxREAL);
        ck(t->h, dcfm_sigma_error(t->h, mxGetDoubles(U), (int32_t)mxGetN(U), sv, (int32_t)it, 1,
                                  mxGetDoubles(plhs[0])));
    } else if (!strcmp(cmd, "set_trace")) {
        nargs(nrhs, 3, cmd);
        slot *t = get(prhs[1]);
        const double cap = scalar(prhs[2], "cap");
        if (cap < 0) mexErrMsgIdAndTxt("dcfm:arg", "cap must be >= 0");
        ck(t->h, dcfm_set_trace(t->h, (int64_t)cap));
    } else if (!strcmp(cmd, "get_trace")) {          /* count x 4, MATLAB column-major */
        nargs(nrhs, 2, cmd);
        slot *t = get(prhs[1]);
        int64_t cnt = 0;
        ck(t->h, dcfm_get_trace(t->h, NULL, &cnt));
        double *rows = (double *)mxMalloc((size_t)(cnt > 0 ? cnt : 1) * 4 * sizeof(double));
        ck(t->h, dcfm_get_trace(t->h, rows, &cnt));
        plhs[0] = mxCreateDoubleMatrix((mwSize)cnt, 4, mxREAL);
        double *o = mxGetDoubles(plhs[0]);
        for (int64_t r = 0; r < cnt; ++r)
            for (int q = 0; q < 4; ++q) o[r + cnt * q] = rows[r * 4 + q];
        mxFree(rows);
    } else if (!strcmp(cmd, "run")) {
        nargs(nrhs, 4, cmd);
        slot *t = get(prhs[1]);
        const double first = scalar(prhs[2], "first"), count = scalar(prhs[3], "count");
        if (first < 1 || count < 0 || first != (double)(int64_t)first || count != (double)(int64_t)count)
            mexErrMsgIdAndTxt("dcfm:arg", "first >= 1 and count >= 0 must be integers");
        ck(t->h, dcfm_run(t->h, (int64_t)first, (int64_t)count));
    } else if (!strcmp(cmd, "get_sigma")) {          /* Sigmaout = dcfm_mex('get_sigma', h) */
        if (nrhs != 2 && nrhs != 3) nargs(nrhs, 2, cmd);
        slot *t = get(prhs[1]);
        const int64_t p = t->P * t->g;               /* the size the library writes */
        if (nrhs == 3 && scalar(prhs[2], "p") != (double)p)
            mexErrMsgIdAndTxt("dcfm:arg", "p = %g does not match the handle's P*g = %lld", mxGetScalar(prhs[2]),
                              (long long)p);
        plhs[0] = mxCreateDoubleMatrix((mwSize)p, (mwSize)p, mxREAL);
        ck(t->h, dcfm_get_sigma(t->h, mxGetDoubles(plhs[0])));
    } else if (!strcmp(cmd, "destroy")) {
        nargs(nrhs, 2, cmd);
        slot *t = get(prhs[1]);
        dcfm_destroy(t->h);
        t->h = 0;
        mexUnlock();
    } else {
        mexErrMsgIdAndTxt("dcfm:cmd", "unknown command %s", cmd);
    }
}
