// copy_probe.hip -- tuning tool (not product code): is the product layout's
// copy rate (9 component planes per layer, 516 x 516 planes of 544-double rows,
// gcmx.hip) below a flat copy of the same bytes, and does the component plane
// stride matter (HBM channel mapping of the 9 + 9 concurrent streams)?
//   flat      : 9*512^3 doubles, contiguous, double2 per lane
//   layout P  : 9 loads + 9 stores per node, one z row per 512-thread block,
//               marching y, component plane stride = CS + P doubles
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
	do {                                                                                \
		hipError_t e = (x);                                                             \
		if (e != hipSuccess) {                                                          \
			std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
			std::exit(1);                                                               \
		}                                                                               \
	} while (0)

constexpr int N = 512, BS = 2, ROW = 544, LEAD = 14;
constexpr long long STY = ROW, STX = (long long)ROW * (N + 2 * BS);
constexpr long long CS = ((STX * (N + 2 * BS)) + 63) / 64 * 64;
constexpr long long ORIGIN = LEAD + BS + BS * STY + BS * STX;
typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_flat(const d2* __restrict__ in, d2* __restrict__ out, long long n2) {
	const long long stride = (long long)gridDim.x * blockDim.x;
	for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride)
		__builtin_nontemporal_store(in[i], out + i);
}

// flat-copy variants for the yardstick (gcmx_copy_ceiling): U loads in flight
// per lane before their stores, non-temporal (NT) or plain stores, nt loads (NTL)
template <int U, bool NT, bool NTL>
__global__ __launch_bounds__(256) void k_flat_u(const d2* __restrict__ in, d2* __restrict__ out, long long n2) {
	const long long nth = (long long)gridDim.x * blockDim.x;
	long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	for (; i + (U - 1) * nth < n2; i += U * nth) {
		d2 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) v[u] = NTL ? __builtin_nontemporal_load(in + i + u * nth) : in[i + u * nth];
#pragma unroll
		for (int u = 0; u < U; u++) {
			if (NT) __builtin_nontemporal_store(v[u], out + i + u * nth);
			else out[i + u * nth] = v[u];
		}
	}
	for (; i < n2; i += nth) out[i] = in[i];
}
// each block copies one contiguous chunk (no grid stride): 256 threads x U x 16 B per step
template <int U>
__global__ __launch_bounds__(256) void k_flat_chunk(const d2* __restrict__ in, d2* __restrict__ out, long long n2,
                                                   long long per_block) {
	const long long b0 = (long long)blockIdx.x * per_block, b1 = min(b0 + per_block, n2);
	for (long long i = b0 + threadIdx.x; i < b1; i += 256 * U) {
		d2 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			if (i + u * 256 < b1) v[u] = in[i + u * 256];
#pragma unroll
		for (int u = 0; u < U; u++)
			if (i + u * 256 < b1) __builtin_nontemporal_store(v[u], out + i + u * 256);
	}
}

// the two halves of a copy alone: U 16-B loads in flight per lane (summed, one
// store per lane that never fires for the zeroed input), or U non-temporal 16-B stores
template <int U>
__global__ __launch_bounds__(256) void k_read_u(const d2* __restrict__ in, d2* __restrict__ out, long long n2) {
	const long long nth = (long long)gridDim.x * blockDim.x;
	long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	d2 acc = {0.0, 0.0};
	for (; i + (U - 1) * nth < n2; i += U * nth) {
		d2 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) v[u] = in[i + u * nth];
#pragma unroll
		for (int u = 0; u < U; u++) acc += v[u];
	}
	for (; i < n2; i += nth) acc += in[i];
	if (acc.x == 1.0e300) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
template <int U>
__global__ __launch_bounds__(256) void k_write_u(d2* __restrict__ out, long long n2, double val) {
	const long long nth = (long long)gridDim.x * blockDim.x;
	long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
	const d2 v = {val, val};
	for (; i + (U - 1) * nth < n2; i += U * nth) {
#pragma unroll
		for (int u = 0; u < U; u++) __builtin_nontemporal_store(v, out + i + u * nth);
	}
	for (; i < n2; i += nth) out[i] = v;
}

__global__ __launch_bounds__(512) void k_layout(const double* __restrict__ in, double* __restrict__ out,
                                                long long cs, int chunk) {
	const int z = threadIdx.x;
	const int T_ = gridDim.x, b = blockIdx.x;
	const int p = (T_ % 8 == 0) ? (b % 8) * (T_ / 8) + b / 8 : b;
	const int x = p % N, yb = (p / N) * chunk;
	const long long base = ORIGIN + x * STX + z;
	for (int y = yb; y < yb + chunk; y++) {
		const long long o = base + (long long)y * STY;
		double v[9];
#pragma unroll
		for (int c = 0; c < 9; c++) v[c] = in[c * cs + o];
#pragma unroll
		for (int c = 0; c < 9; c++) __builtin_nontemporal_store(v[c], out + c * cs + o);
	}
}

template <class F>
float timeit(F launch) {
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	launch();
	CK(hipDeviceSynchronize());
	CK(hipEventRecord(a));
	for (int r = 0; r < 10; r++) launch();
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	return ms / 10;
}

int main() {
	const double nodes = (double)N * N * N;
	const long long maxcs = CS + 8192;
	const size_t bytes = (size_t)9 * maxcs * sizeof(double);
	double *in, *out;
	CK(hipMalloc(&in, bytes));
	CK(hipMalloc(&out, bytes));
	CK(hipMemset(in, 0, bytes));
	CK(hipMemset(out, 0, bytes));
	const long long n2 = (long long)9 * N * N * N / 2;
	for (int g : {2048, 8192, 32768}) {
		float ms = timeit([&] { hipLaunchKernelGGL(k_flat, dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		std::printf("flat copy grid %6d: %.3f ms (%.0f GB/s)\n", g, ms, 144.0 * nodes / (ms * 1e6));
	}
	auto rate = [&](float ms) { return 144.0 * nodes / (ms * 1e6); };
	for (int g : {1024, 2048, 4096, 8192, 16384}) {
		float a = timeit([&] { hipLaunchKernelGGL((k_flat_u<1, true, false>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		float b = timeit([&] { hipLaunchKernelGGL((k_flat_u<4, true, false>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		float c = timeit([&] { hipLaunchKernelGGL((k_flat_u<4, false, false>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		float d = timeit([&] { hipLaunchKernelGGL((k_flat_u<4, true, true>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		float e = timeit([&] { hipLaunchKernelGGL((k_flat_u<8, true, false>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		std::printf("flat grid %6d: U1 nt %.0f  U4 nt %.0f  U4 plain %.0f  U4 nt+ntload %.0f  U8 nt %.0f GB/s\n", g, rate(a),
		            rate(b), rate(c), rate(d), rate(e));
	}
	for (int nb : {2048, 4096, 16384, 65536}) {
		const long long per = (n2 + nb - 1) / nb;
		float a = timeit([&] { hipLaunchKernelGGL((k_flat_chunk<4>), dim3(nb), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2, per); });
		std::printf("chunked %6d blocks (U4, nt stores): %.0f GB/s\n", nb, rate(a));
	}
	// read-only and write-only passes over the same 9.66 GB each: if HBM overlapped
	// a copy's reads and writes perfectly the copy would take max(t_r, t_w); a copy
	// near t_r + t_w means the stack alternates between the two directions
	auto half = [&](float ms) { return 72.0 * nodes / (ms * 1e6); };
	for (int g : {2048, 8192, 16384}) {
		float r4 = timeit([&] { hipLaunchKernelGGL((k_read_u<4>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		float r8 = timeit([&] { hipLaunchKernelGGL((k_read_u<8>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		float w4 = timeit([&] { hipLaunchKernelGGL((k_write_u<4>), dim3(g), dim3(256), 0, 0, (d2*)out, n2, 0.0); });
		float c4 = timeit([&] { hipLaunchKernelGGL((k_flat_u<4, true, false>), dim3(g), dim3(256), 0, 0, (const d2*)in, (d2*)out, n2); });
		std::printf("grid %6d: read-only U4 %.3f ms (%.0f GB/s)  U8 %.3f ms (%.0f GB/s)  write-only U4 %.3f ms (%.0f GB/s)  "
		            "copy U4 %.3f ms (%.0f GB/s; read+write alone %.3f ms)\n",
		            g, r4, half(r4), r8, half(r8), w4, half(w4), c4, rate(c4), (r4 < r8 ? r4 : r8) + w4);
	}
	if (std::getenv("COPY_ONLY")) return 0;
	for (int chunk : {128, 32}) {
		for (long long pad : {0LL, 16LL, 32LL, 48LL, 64LL, 96LL, 160LL, 256LL, 544LL, 1024LL, 2048LL, 4096LL}) {
			const long long cs = CS + pad;
			float ms = timeit([&] {
				hipLaunchKernelGGL(k_layout, dim3((N / chunk) * N), dim3(512), 0, 0, in, out, cs, chunk);
			});
			std::printf("layout copy chunk %3d plane stride CS+%5lld (CS %% 4096 = %4lld doubles): %.3f ms (%.0f GB/s)\n",
			            chunk, pad, cs % 4096, ms, 144.0 * nodes / (ms * 1e6));
		}
	}
	return 0;
}
