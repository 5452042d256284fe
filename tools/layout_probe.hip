// layout_probe.hip -- tuning tool (not product code): the two-planes-per-thread
// access pattern of k_step_tx2 (6 components at x-2..x+3, 3 at x and x+1, 9
// stores at x and x+1, marching y, one block per plane pair and 128-row chunk,
// XCD-aware order) in two device layouts of the same 512^3 bs-2 grid:
//   soa : component planes 1.1 GB apart (the product layout, gcmx.hip)
//   row : components interleaved per padded row, [x][y][c][z] (each block row
//         reads 9 consecutive 4.3 KB rows per plane)
// plus the plain 9-in/9-out copy in both, with trivial arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/layout_probe tools/layout_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
	do {                                                                    \
		hipError_t e = (x);                                                 \
		if (e != hipSuccess) {                                              \
			std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));     \
			std::exit(1);                                                   \
		}                                                                   \
	} while (0)

constexpr int N = 512, BS = 2, ROW = 544, LEAD = 14, NA = N + 2 * BS;
// element index of (x, y, c, z) in inner coordinates; x, y may be ghosts (>= -BS)
template <bool ROWI>
__device__ __forceinline__ long long idx(int x, int y, int c, int z) {
	const long long X = x + BS, Y = y + BS, Z = z + LEAD + BS;
	if constexpr (ROWI) return ((X * NA + Y) * 9 + c) * ROW + Z;
	else return (long long)c * ((long long)NA * NA * ROW + 64) + (X * NA + Y) * ROW + Z;
}

template <bool ROWI, bool XPAT>
__global__ __launch_bounds__(512, 2) void k_probe(const double* __restrict__ in, double* __restrict__ out,
                                                  int chunk) {
	const int z = threadIdx.x;
	const int T = gridDim.x, b = blockIdx.x;
	const int p = (T % 8 == 0) ? (b % 8) * (T / 8) + b / 8 : b;
	const int np = N / 2;
	const int x = (p % np) * 2, yb = (p / np) * chunk;
	for (int y = yb; y < yb + chunk; y++) {
		double v[2][9];
#pragma unroll
		for (int c = 0; c < 9; c++) {
			if (XPAT && c < 6) {
				double w[6];
#pragma unroll
				for (int k = 0; k < 6; k++) w[k] = in[idx<ROWI>(x - 2 + k, y, c, z)];
#pragma unroll
				for (int t = 0; t < 2; t++) v[t][c] = w[t] + w[t + 1] + w[t + 2] + w[t + 3] + w[t + 4];
			} else {
#pragma unroll
				for (int t = 0; t < 2; t++) v[t][c] = in[idx<ROWI>(x + t, y, c, z)];
			}
		}
#pragma unroll
		for (int t = 0; t < 2; t++)
#pragma unroll
			for (int c = 0; c < 9; c++) __builtin_nontemporal_store(v[t][c], &out[idx<ROWI>(x + t, y, c, z)]);
	}
}

template <bool ROWI, bool XPAT>
float run(const double* in, double* out, int reps) {
	const int chunk = 128;
	dim3 grid((N / chunk) * (N / 2));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	hipLaunchKernelGGL((k_probe<ROWI, XPAT>), grid, dim3(512), 0, 0, in, out, chunk);
	CK(hipDeviceSynchronize());
	CK(hipEventRecord(a));
	for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_probe<ROWI, XPAT>), grid, dim3(512), 0, 0, in, out, chunk);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	return ms / reps;
}

int main() {
	const size_t elems = (size_t)9 * ((size_t)NA * NA * ROW + 64);
	double *in, *out;
	CK(hipMalloc(&in, elems * sizeof(double)));
	CK(hipMalloc(&out, elems * sizeof(double)));
	CK(hipMemset(in, 0, elems * sizeof(double)));
	CK(hipMemset(out, 0, elems * sizeof(double)));
	const double nodes = (double)N * N * N;
	for (int rep = 0; rep < 2; rep++) {
		const float c0 = run<false, false>(in, out, 10), c1 = run<true, false>(in, out, 10);
		const float x0 = run<false, true>(in, out, 10), x1 = run<true, true>(in, out, 10);
		std::printf("copy  soa %.3f ms (%.0f GB/s)  row %.3f ms (%.0f GB/s)\n", c0, 144.0 * nodes / (c0 * 1e6), c1,
		            144.0 * nodes / (c1 * 1e6));
		std::printf("tx2   soa %.3f ms (%.0f GB/s)  row %.3f ms (%.0f GB/s)\n", x0, 144.0 * nodes / (x0 * 1e6), x1,
		            144.0 * nodes / (x1 * 1e6));
	}
	return 0;
}
