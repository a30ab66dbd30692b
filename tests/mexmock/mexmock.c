/*
 * mexmock.c — mock MEX runtime for tests/test_mex_gateway.py (test infrastructure, not
 * MATLAB): mxArrays as plain heap objects, mexErrMsgIdAndTxt as a longjmp back to mm_call,
 * and mm_* helpers that ctypes uses to build arguments and read results.
 */
#include "mex.h"
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct mxArray_tag {
    mxClassID cls;
    int cplx;
    size_t ndim, dims[8];
    void *data;                 /* numeric data, or the char string */
    size_t nfields;
    char **fnames;
    mxArray **fvals;
};

static jmp_buf *g_jb;
static char g_id[128], g_msg[4096];
static void (*g_exit)(void);
static int g_locks;

static size_t numel(const mxArray *a) {
    size_t n = 1;
    for (size_t d = 0; d < a->ndim; ++d) n *= a->dims[d];
    return n;
}
static size_t esize(mxClassID c) {
    switch (c) {
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    case mxSINGLE_CLASS: case mxINT32_CLASS: case mxUINT32_CLASS: return 4;
    case mxINT16_CLASS: case mxUINT16_CLASS: case mxCHAR_CLASS: return 2;
    default: return 1;
    }
}
static mxArray *alloc(mxClassID cls, size_t ndim, const size_t *dims) {
    mxArray *a = calloc(1, sizeof *a);
    a->cls = cls;
    a->ndim = ndim < 2 ? 2 : ndim;
    a->dims[0] = a->dims[1] = 1;
    for (size_t d = 0; d < ndim && d < 8; ++d) a->dims[d] = dims[d];
    a->data = calloc(numel(a) ? numel(a) : 1, esize(cls));
    return a;
}

/* ---- MEX / mx API ---------------------------------------------------------------- */
void mexErrMsgIdAndTxt(const char *errorid, const char *errormsg, ...) {
    va_list ap;
    va_start(ap, errormsg);
    snprintf(g_id, sizeof g_id, "%s", errorid);
    vsnprintf(g_msg, sizeof g_msg, errormsg, ap);
    va_end(ap);
    if (g_jb) longjmp(*g_jb, 1);
    fprintf(stderr, "mexmock: error outside mm_call: %s: %s\n", g_id, g_msg);
    abort();
}
int mexAtExit(void (*f)(void)) { g_exit = f; return 0; }
void mexLock(void) { ++g_locks; }
void mexUnlock(void) { --g_locks; }

mxArray *mxGetField(const mxArray *pm, mwIndex index, const char *name) {
    if (!pm || pm->cls != mxSTRUCT_CLASS || index != 0) return NULL;
    for (size_t f = 0; f < pm->nfields; ++f)
        if (!strcmp(pm->fnames[f], name)) return pm->fvals[f];
    return NULL;
}
double mxGetScalar(const mxArray *pm) {
    if (!numel(pm)) return 0.0;
    switch (pm->cls) {
    case mxDOUBLE_CLASS: return ((double *)pm->data)[0];
    case mxINT64_CLASS: return (double)((int64_t *)pm->data)[0];
    default: return 0.0;
    }
}
bool mxIsDouble(const mxArray *pm) { return pm->cls == mxDOUBLE_CLASS; }
bool mxIsComplex(const mxArray *pm) { return pm->cplx != 0; }
bool mxIsChar(const mxArray *pm) { return pm->cls == mxCHAR_CLASS; }
bool mxIsStruct(const mxArray *pm) { return pm->cls == mxSTRUCT_CLASS; }
bool mxIsInt64(const mxArray *pm) { return pm->cls == mxINT64_CLASS; }
size_t mxGetNumberOfElements(const mxArray *pm) { return numel(pm); }
size_t mxGetM(const mxArray *pm) { return pm->dims[0]; }
size_t mxGetN(const mxArray *pm) {
    size_t n = 1;
    for (size_t d = 1; d < pm->ndim; ++d) n *= pm->dims[d];
    return n;
}
int mxGetString(const mxArray *pm, char *str, mwSize len) {
    if (pm->cls != mxCHAR_CLASS || len == 0) return 1;
    const char *s = (const char *)pm->data;
    const size_t n = strlen(s);
    snprintf(str, len, "%s", s);
    return n + 1 > len;
}
mxDouble *mxGetDoubles(const mxArray *pa) { return pa->cls == mxDOUBLE_CLASS && !pa->cplx ? pa->data : NULL; }
mxInt64 *mxGetInt64s(const mxArray *pa) { return pa->cls == mxINT64_CLASS ? pa->data : NULL; }
mxArray *mxCreateDoubleScalar(double v) {
    const size_t one[2] = {1, 1};
    mxArray *a = alloc(mxDOUBLE_CLASS, 2, one);
    ((double *)a->data)[0] = v;
    return a;
}
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity flag) {
    const size_t d[2] = {m, n};
    mxArray *a = alloc(mxDOUBLE_CLASS, 2, d);
    a->cplx = flag == mxCOMPLEX;
    return a;
}
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID cls, mxComplexity flag) {
    mxArray *a = alloc(cls, ndim, dims);
    a->cplx = flag == mxCOMPLEX;
    return a;
}
void mxDestroyArray(mxArray *pm) {
    if (!pm) return;
    for (size_t f = 0; f < pm->nfields; ++f) {
        free(pm->fnames[f]);
        mxDestroyArray(pm->fvals[f]);
    }
    free(pm->fnames);
    free(pm->fvals);
    free(pm->data);
    free(pm);
}
void *mxMalloc(mwSize n) { return malloc(n ? n : 1); }
void mxFree(void *p) { free(p); }

/* ---- helpers for the ctypes driver ------------------------------------------------ */
mxArray *mm_numeric(int cls, int ndim, const int64_t *dims, const void *data, int cplx) {
    size_t d[8];
    for (int i = 0; i < ndim && i < 8; ++i) d[i] = (size_t)dims[i];
    mxArray *a = alloc((mxClassID)cls, (size_t)ndim, d);
    a->cplx = cplx;
    if (data) memcpy(a->data, data, numel(a) * esize(a->cls));
    return a;
}
mxArray *mm_string(const char *s) {
    const size_t d[2] = {1, strlen(s)};
    mxArray *a = alloc(mxCHAR_CLASS, 2, d);
    free(a->data);
    a->data = strdup(s);
    return a;
}
/* takes ownership of vals */
mxArray *mm_struct(int nf, const char **names, mxArray **vals) {
    const size_t one[2] = {1, 1};
    mxArray *a = alloc(mxSTRUCT_CLASS, 2, one);
    a->nfields = (size_t)nf;
    a->fnames = calloc((size_t)nf + 1, sizeof(char *));
    a->fvals = calloc((size_t)nf + 1, sizeof(mxArray *));
    for (int f = 0; f < nf; ++f) {
        a->fnames[f] = strdup(names[f]);
        a->fvals[f] = vals[f];
    }
    return a;
}
void *mm_data(mxArray *a) { return a->data; }
int64_t mm_numel(const mxArray *a) { return (int64_t)numel(a); }
int mm_ndim(const mxArray *a) { return (int)a->ndim; }
int64_t mm_dim(const mxArray *a, int d) { return d < (int)a->ndim ? (int64_t)a->dims[d] : 1; }
void mm_free(mxArray *a) { mxDestroyArray(a); }
/* 0: returned normally, 1: raised (mm_error_id / mm_error_msg) */
int mm_call(int nlhs, mxArray **plhs, int nrhs, const mxArray **prhs) {
    jmp_buf jb;
    g_id[0] = g_msg[0] = 0;
    if (setjmp(jb)) {
        g_jb = NULL;
        return 1;
    }
    g_jb = &jb;
    mexFunction(nlhs, plhs, nrhs, prhs);
    g_jb = NULL;
    return 0;
}
const char *mm_error_id(void) { return g_id; }
const char *mm_error_msg(void) { return g_msg; }
int mm_locks(void) { return g_locks; }
void mm_exit(void) { if (g_exit) g_exit(); }
