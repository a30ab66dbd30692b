/* Malformed-call suite of the MEX gateway (matlab/dcfm_mex.c) as a standalone program, so the
 * gateway and the mock runtime can be built with -fsanitize=address,undefined (test
 * infrastructure; tests/test_mex_gateway.py builds and runs it).  Every call below must be
 * rejected by the gateway with the expected error id before the library reads a pointer;
 * the sanitizers abort on any out-of-bounds access, use after free or undefined behaviour on
 * the way.  Prints "ok" and exits 0 when every case behaved. */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "mex.h"

mxArray *mm_numeric(int cls, int ndim, const int64_t *dims, const void *data, int cplx);
mxArray *mm_string(const char *s);
mxArray *mm_struct(int nf, const char **names, mxArray **vals);
void mm_free(mxArray *a);
int mm_call(int nlhs, mxArray **plhs, int nrhs, const mxArray **prhs);
const char *mm_error_id(void);
int mm_locks(void);

static int failures = 0;

static mxArray *scalar(double v) {
    const int64_t dims[2] = {1, 1};
    return mm_numeric(6 /* mxDOUBLE_CLASS */, 2, dims, &v, 0);
}
static mxArray *vec(int n, double v) {
    double buf[8];
    for (int i = 0; i < n && i < 8; ++i) buf[i] = v;
    const int64_t dims[2] = {n, 1};
    return mm_numeric(6, 2, dims, buf, 0);
}
static mxArray *cfg(const char *override, mxArray *value) {
    const char *names[9] = {"n", "P", "g", "K", "rho", "burnin", "mcmc", "thin", "inject"};
    const double vals[9] = {30, 10, 4, 3, 0.5, 1, 2, 1, 1};
    mxArray *v[9];
    for (int i = 0; i < 9; ++i)
        v[i] = (override && !strcmp(override, names[i])) ? value : scalar(vals[i]);
    return mm_struct(9, names, v);
}
/* call the gateway, expect failure with error id `want` */
static void expect(const char *what, const char *want, int nrhs, mxArray **args) {
    mxArray *out[2] = {NULL, NULL};
    const int rc = mm_call(1, out, nrhs, (const mxArray **)args);
    const char *id = mm_error_id();
    if (rc == 0 || !id || strcmp(id, want) != 0) {
        fprintf(stderr, "%s: expected %s, got rc %d id %s\n", what, want, rc, id ? id : "(none)");
        ++failures;
    }
    for (int i = 0; i < 2; ++i)
        if (out[i]) mm_free(out[i]);
    for (int i = 0; i < nrhs; ++i) mm_free(args[i]);
}

int main(void) {
    {   mxArray *a[1] = {scalar(3.0)}; expect("command not a string", "dcfm:cmd", 1, a); }
    {   mxArray *a[1] = {mm_string("frobnicate")}; expect("unknown command", "dcfm:cmd", 1, a); }
    {   mxArray *a[1] = {mm_string("create")}; expect("create without cfg", "dcfm:nargs", 1, a); }
    {   mxArray *a[2] = {mm_string("create"), scalar(1.0)}; expect("cfg not a struct", "dcfm:cfg", 2, a); }
    {   mxArray *a[2] = {mm_string("create"), cfg("rho", vec(2, 0.5))}; expect("non-scalar field", "dcfm:cfg", 2, a); }
    {   mxArray *a[2] = {mm_string("create"), cfg("rho", scalar(1.5))}; expect("rho outside [0,1]", "dcfm:create", 2, a); }
    {   mxArray *a[2] = {mm_string("create"), cfg("K", scalar(0.0))}; expect("K = 0", "dcfm:create", 2, a); }
    {   mxArray *a[2] = {mm_string("create"), cfg("thin", scalar(0.0))}; expect("thin = 0", "dcfm:create", 2, a); }
    {   mxArray *a[4] = {mm_string("run"), scalar(7.0), scalar(1.0), scalar(1.0)}; expect("run: bad handle", "dcfm:handle", 4, a); }
    {   mxArray *a[2] = {mm_string("get_sigma"), scalar(7.0)}; expect("get_sigma: bad handle", "dcfm:handle", 2, a); }
    {   mxArray *a[3] = {mm_string("set_data"), scalar(7.0), vec(3, 0.0)}; expect("set_data: bad handle", "dcfm:handle", 3, a); }
    {   mxArray *a[2] = {mm_string("destroy"), scalar(7.0)}; expect("destroy: bad handle", "dcfm:handle", 2, a); }
    if (mm_locks() != 0) {
        fprintf(stderr, "mexLock count %d after rejected calls\n", mm_locks());
        ++failures;
    }
    if (failures) return 1;
    printf("ok\n");
    return 0;
}
