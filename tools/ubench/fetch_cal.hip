// FETCH_SIZE calibration for the access widths of the x3 dgrad's loads (MI355X_MICROARCH.md: FETCH_SIZE
// reads half the bytes of a 16-B-per-lane streaming read; other widths are uncalibrated). Each kernel
// reads every byte of a 1 GiB buffer (4x the Infinity Cache) exactly once and writes one word per
// workgroup; run each under rocprofv3 --pmc FETCH_SIZE and divide by the bytes read.
//   w16: 16 B/lane, contiguous                 (x / bit-map LDS-DMA, act16 images)
//   w4:  4 B/lane, contiguous
//   dy4: 4 B/lane in the dgrad's load_dy pattern: lanes 8g..8g+7 = 8 consecutive floats, g = segment of
//        a different 4-channel group (stride 576 B = 4 x 144 floats), 4 channels per lane
//   dy1: the same pattern over uint8 (the routing codes)
// usage: fetch_cal <w16|w4|dy4|dy1>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
constexpr size_t NB = 1ull << 30;
__global__ void w16(const uint4* p, size_t n, unsigned* out) {
    unsigned s = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) { uint4 v = p[i]; s ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (s == 0x12345678u) out[blockIdx.x] = s;
}
__global__ void w4(const unsigned* p, size_t n, unsigned* out) {
    unsigned s = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) s ^= p[i];
    if (s == 0x12345678u) out[blockIdx.x] = s;
}
// element e of a "sample" of 64 channels x 144 windows: 16 channel groups x 144 windows = 2304 items of
// 4 channels; item i: channel group c4 = i & 7 (+8 for the second half), window wi = i >> 3 like load_dy
template <typename T>
__global__ void dy(const T* p, size_t nsamples, unsigned* out) {
    unsigned s = 0;
    const int tid = threadIdx.x;
    for (size_t b = blockIdx.x; b < nsamples; b += gridDim.x) {
        const T* base = p + b * 9216;
        for (int it = tid; it < 2 * 1152; it += 256) {
            const int h = it / 1152, i = it % 1152;
            const int c4 = i & 7, wi = i >> 3;
            const size_t o = (size_t)(32 * h + 4 * c4) * 144 + wi;
#pragma unroll
            for (int j = 0; j < 4; ++j) s ^= (unsigned)base[o + j * 144];
        }
    }
    if (s == 0x12345678u) out[blockIdx.x] = s;
}
int main(int argc, char** argv) {
    const char* k = argc > 1 ? argv[1] : "w16";
    void* buf; unsigned* out;
    if (hipMalloc(&buf, NB) != hipSuccess || hipMalloc(&out, 4096 * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, NB);
    for (int rep = 0; rep < 3; ++rep) {
        if (!strcmp(k, "w16")) w16<<<2048, 256>>>((const uint4*)buf, NB / 16, out);
        else if (!strcmp(k, "w4")) w4<<<2048, 256>>>((const unsigned*)buf, NB / 4, out);
        else if (!strcmp(k, "dy4")) dy<float><<<2048, 256>>>((const float*)buf, NB / (9216 * 4), out);
        else dy<unsigned char><<<2048, 256>>>((const unsigned char*)buf, NB / 9216, out);
    }
    (void)hipDeviceSynchronize();
    const double bytes = !strcmp(k, "dy4") ? (double)(NB / (9216 * 4)) * 9216 * 4 : !strcmp(k, "dy1") ? (double)(NB / 9216) * 9216 : (double)NB;
    printf("%s bytes_read_per_launch %.0f\n", k, bytes);
    return 0;
}
