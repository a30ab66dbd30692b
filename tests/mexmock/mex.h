/*
 * mex.h — a minimal stand-in for MATLAB's MEX / matrix API (interleaved-complex API,
 * -R2018a), declaring only what matlab/dcfm_mex.c calls, with the documented signatures.
 * Test infrastructure: lets the gateway be compiled with gcc and driven through the mock
 * runtime in mexmock.c (tests/test_mex_gateway.py).  Not MATLAB.
 */
#ifndef DCFM_MEXMOCK_H
#define DCFM_MEXMOCK_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

typedef size_t mwSize;
typedef size_t mwIndex;
typedef double mxDouble;
typedef int64_t mxInt64;
typedef struct mxArray_tag mxArray;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef enum {
    mxUNKNOWN_CLASS = 0, mxCELL_CLASS, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxVOID_CLASS,
    mxDOUBLE_CLASS, mxSINGLE_CLASS, mxINT8_CLASS, mxUINT8_CLASS, mxINT16_CLASS, mxUINT16_CLASS,
    mxINT32_CLASS, mxUINT32_CLASS, mxINT64_CLASS, mxUINT64_CLASS
} mxClassID;

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]);

void mexErrMsgIdAndTxt(const char *errorid, const char *errormsg, ...) __attribute__((noreturn));
int mexAtExit(void (*ExitFcn)(void));
void mexLock(void);
void mexUnlock(void);

mxArray *mxGetField(const mxArray *pm, mwIndex index, const char *fieldname);
double mxGetScalar(const mxArray *pm);
bool mxIsDouble(const mxArray *pm);
bool mxIsComplex(const mxArray *pm);
bool mxIsChar(const mxArray *pm);
bool mxIsStruct(const mxArray *pm);
bool mxIsInt64(const mxArray *pm);
size_t mxGetNumberOfElements(const mxArray *pm);
size_t mxGetM(const mxArray *pm);
size_t mxGetN(const mxArray *pm);
int mxGetString(const mxArray *pm, char *str, mwSize strlen);
mxDouble *mxGetDoubles(const mxArray *pa);
mxInt64 *mxGetInt64s(const mxArray *pa);
mxArray *mxCreateDoubleScalar(double value);
mxArray *mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity flag);
mxArray *mxCreateNumericArray(mwSize ndim, const mwSize *dims, mxClassID classid, mxComplexity flag);
void mxDestroyArray(mxArray *pm);
void *mxMalloc(mwSize n);
void mxFree(void *ptr);
#endif
