"""Dev instrumentation (never shipped): per-block start / end s_memrealtime stamps of the last
k_wcol launch, read back with dcfm_debug_stamps (tools/stamps.py)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = """__global__ __launch_bounds__(256) void k_wcol(Dims d, Bufs b, int ops, int colsum, int wpass,
                                              unsigned long long ops_epoch, int xchol) {"""
assert old in s
s = s.replace(old, """__device__ unsigned long long g_stamp[8192][2];
__device__ __forceinline__ void wcol_body(Dims d, Bufs b, int ops, int colsum, int wpass, unsigned long long ops_epoch,
                                          int xchol, double *smem);
__global__ __launch_bounds__(256) void k_wcol(Dims d, Bufs b, int ops, int colsum, int wpass,
                                              unsigned long long ops_epoch, int xchol) {
    __shared__ double smem_[PREP_SMEM];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    wcol_body(d, b, ops, colsum, wpass, ops_epoch, xchol, smem_);
    __syncthreads();
    if (wpass && threadIdx.x == 0 && blockIdx.x < 8192) {
        g_stamp[blockIdx.x][0] = t0;
        g_stamp[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
    }
}
__device__ __forceinline__ void wcol_body(Dims d, Bufs b, int ops, int colsum, int wpass, unsigned long long ops_epoch,
                                          int xchol, double *smem) {""", 1)
# the body's own shared array becomes the passed pointer
old2 = """                                          int xchol, double *smem) {
    __shared__ double smem[PREP_SMEM];"""
assert old2 in s
s = s.replace(old2, """                                          int xchol, double *smem) {""")
s = s.replace("void launch_wcol(const Dims &d,", """}  // namespace dcfm
extern "C" int dcfm_debug_stamps(unsigned long long *out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(dcfm::g_stamp), (size_t)n * 2 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
namespace dcfm {
void launch_wcol(const Dims &d,""", 1)
open(f, "w").write(s)
