// calib_fetch.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access widths
// the gcmx kernels use (8-byte loads/stores per lane, 64 lanes = 512 B per
// wave-instruction).  MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a
// 16-B/lane stream on gfx950 and other widths are uncalibrated, so this program
// streams a known byte count with each width; rocprofv3 --pmc gives the ratio.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read8(const double* __restrict__ a, double* __restrict__ out, long long n) {
	double acc = 0;
	for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
		acc += a[i];
	if (acc == 12345.678) out[0] = acc;  // keep the loads
}
__global__ void read16(const double2* __restrict__ a, double* __restrict__ out, long long n) {
	double acc = 0;
	for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
		double2 v = a[i];
		acc += v.x + v.y;
	}
	if (acc == 12345.678) out[0] = acc;
}
__global__ void write8(double* __restrict__ a, long long n) {
	for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
		a[i] = (double)i;
}

int main() {
	const long long n = 1LL << 30;  // 8 GiB of doubles: far beyond the 256 MiB Infinity Cache
	double *a, *out;
	if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
	hipMemset(a, 0, n * 8);
	for (int r = 0; r < 2; r++) {
		write8<<<8192, 256>>>(a, n);
		read8<<<8192, 256>>>(a, out, n);
		read16<<<8192, 256>>>((const double2*)a, out, n / 2);
	}
	if (hipDeviceSynchronize() != hipSuccess) return 2;
	printf("calib: each launch moves %lld bytes\n", n * 8);
	hipFree(a);
	hipFree(out);
	return 0;
}
