// A non-Python host for the detector call of torch_models/detect.py:78: plain C++ against
// include/edgedet.h and the HIP runtime, no Python, no torch.  It reads a packed weight blob
// (edgedet_model_pack output) and a raw image batch, runs edgedet_model_forward, and writes the
// detections as raw arrays — the same call sequence a Go (cgo), Java (JNI) or Node (N-API) binding
// makes.
//
//   native_host KIND NUM_CLASSES REDUCED_TAIL B H W U8 WEIGHTS.bin IMAGES.bin OUT_PREFIX
//     KIND 0 = SSDLite, 1 = Faster R-CNN; IMAGES.bin = B x 3 x H x W (uint8 if U8 else float32)
//   writes OUT_PREFIX.count (int32 [B]), .boxes (float32 [B][K][4]), .scores (float32 [B][K]),
//   .labels (int64 [B][K])
//
// Build: hipcc -O2 tools/native_host.cpp -Iinclude -Ledgeml-object-detection_amd -ledgedet \
//        -Wl,-rpath,'$ORIGIN/../edgeml-object-detection_amd' -o tools/native_host
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "edgedet.h"

#define CK(e)                                                                               \
    do {                                                                                    \
        hipError_t r_ = (e);                                                                \
        if (r_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_));       \
            return 3;                                                                       \
        }                                                                                   \
    } while (0)
#define ED(e)                                                                               \
    do {                                                                                    \
        int r_ = (int)(e);                                                                  \
        if (r_ != 0) {                                                                      \
            fprintf(stderr, "%s:%d edgedet error %d: %s\n", __FILE__, __LINE__, r_, edgedet_last_error()); \
            return 4;                                                                       \
        }                                                                                   \
    } while (0)

static std::vector<char> slurp(const char* path) {
    std::vector<char> v;
    FILE* f = fopen(path, "rb");
    if (!f) return v;
    fseek(f, 0, SEEK_END);
    v.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(v.data(), 1, v.size(), f) != v.size()) v.clear();
    fclose(f);
    return v;
}

static int spit(const std::string& path, const void* p, size_t n) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f || fwrite(p, 1, n, f) != n) return 1;
    return fclose(f);
}

int main(int argc, char** argv) {
    if (argc != 11) {
        fprintf(stderr, "usage: %s KIND NUM_CLASSES REDUCED_TAIL B H W U8 WEIGHTS.bin IMAGES.bin OUT_PREFIX\n", argv[0]);
        return 2;
    }
    const int kind = atoi(argv[1]), nc = atoi(argv[2]), rt = atoi(argv[3]);
    const int B = atoi(argv[4]), H = atoi(argv[5]), W = atoi(argv[6]), u8 = atoi(argv[7]);
    std::vector<char> wts = slurp(argv[8]), imgs = slurp(argv[9]);
    const int64_t wbytes = edgedet_model_weights_size(kind, nc, rt);
    const size_t ibytes = (size_t)B * 3 * H * W * (u8 ? 1 : 4);
    if (wbytes < 0 || (int64_t)wts.size() != wbytes || imgs.size() != ibytes) {
        fprintf(stderr, "bad inputs: weights %zu (want %lld), images %zu (want %zu): %s\n", wts.size(),
                (long long)wbytes, imgs.size(), ibytes, edgedet_last_error());
        return 2;
    }
    const int64_t ws_bytes = edgedet_model_workspace_size(kind, nc, rt, B, H, W, u8);
    const int K = edgedet_model_max_detections(kind);
    if (ws_bytes < 0 || K <= 0) {
        fprintf(stderr, "edgedet: %s\n", edgedet_last_error());
        return 4;
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void *d_w, *d_x, *d_ws, *d_count, *d_boxes, *d_scores, *d_labels;
    CK(hipMalloc(&d_w, (size_t)wbytes));
    CK(hipMalloc(&d_x, ibytes));
    CK(hipMalloc(&d_ws, (size_t)ws_bytes));
    CK(hipMalloc(&d_count, (size_t)B * 4));
    CK(hipMalloc(&d_boxes, (size_t)B * K * 16));
    CK(hipMalloc(&d_scores, (size_t)B * K * 4));
    CK(hipMalloc(&d_labels, (size_t)B * K * 8));
    CK(hipMemcpy(d_w, wts.data(), (size_t)wbytes, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, imgs.data(), ibytes, hipMemcpyHostToDevice));
    ED(edgedet_model_prepare(kind, nc, rt, B, H, W, u8, d_ws, s));
    ED(edgedet_model_forward(kind, nc, rt, d_w, d_x, B, H, W, u8, d_ws, (int32_t*)d_count, (float*)d_boxes,
                             (float*)d_scores, (int64_t*)d_labels, s));
    CK(hipStreamSynchronize(s));
    std::vector<char> count((size_t)B * 4), boxes((size_t)B * K * 16), scores((size_t)B * K * 4), labels((size_t)B * K * 8);
    CK(hipMemcpy(count.data(), d_count, count.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(boxes.data(), d_boxes, boxes.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(scores.data(), d_scores, scores.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(labels.data(), d_labels, labels.size(), hipMemcpyDeviceToHost));
    const std::string o = argv[10];
    if (spit(o + ".count", count.data(), count.size()) || spit(o + ".boxes", boxes.data(), boxes.size()) ||
        spit(o + ".scores", scores.data(), scores.size()) || spit(o + ".labels", labels.data(), labels.size()))
        return 5;
    for (void* p : {d_w, d_x, d_ws, d_count, d_boxes, d_scores, d_labels}) CK(hipFree(p));
    CK(hipStreamDestroy(s));
    printf("native_host: %d images, %lld workspace bytes, detections per image:", B, (long long)ws_bytes);
    for (int b = 0; b < B; ++b) printf(" %d", ((int32_t*)count.data())[b]);
    printf("\n");
    return 0;
}
