/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked or loaded by the product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *
 * Plain-C restatement of the two torchvision CPU operators that sit on the
 * detection hot path of the reference (torch_models/detect.py:78 reaches them
 * through torchvision.models.detection):
 *
 *   - nms_ref:       torchvision::nms CPU kernel (greedy, stable score sort,
 *                    suppress when inter/(area_i+area_j-inter) > thr, fp32 math,
 *                    threshold compared in double).
 *                    Used by batched_nms at SSD postprocess,
 *                    RPN filter_proposals (A.2 step 4) and RoIHeads (A.2 step 7).
 *   - roi_align_ref: torchvision::roi_align CPU forward, aligned=False
 *                    (SURVEY A.2 step 5), with pre-computed bilinear weights
 *                    exactly as the reference's pre_calc_for_bilinear_interpolate.
 *                    Input here is NCHW like the reference.
 *
 * torchvision is a third-party dependency absent from /root/reference
 * (unpinned version, >=0.13 per the weights= API used at
 * detect.py:24,30).  This file restates its published algorithm.  Compile with
 * -ffp-contract=off so every product/sum rounds separately as in the
 * reference's scalar C++ loops.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* stable descending order of scores (ties keep the lower index first) */
static const float* g_sort_scores;
static int cmp_desc_stable(const void* a, const void* b) {
    int ia = *(const int*)a, ib = *(const int*)b;
    float sa = g_sort_scores[ia], sb = g_sort_scores[ib];
    if (sa > sb) return -1;
    if (sa < sb) return 1;
    return (ia < ib) ? -1 : (ia > ib);
}

/*
 * boxes: [n,4] xyxy fp32; scores [n]; keep_out: [n] int64 indices in kept order.
 * returns number kept.
 */
int64_t nms_ref(const float* boxes, const float* scores, int64_t n, double iou_threshold,
                int64_t* keep_out) {
    if (n <= 0) return 0;
    int* order = (int*)malloc(sizeof(int) * n);
    float* areas = (float*)malloc(sizeof(float) * n);
    unsigned char* suppressed = (unsigned char*)calloc(n, 1);
    for (int64_t i = 0; i < n; i++) {
        order[i] = (int)i;
        float w = boxes[4 * i + 2] - boxes[4 * i + 0];
        float h = boxes[4 * i + 3] - boxes[4 * i + 1];
        areas[i] = w * h;
    }
    g_sort_scores = scores;
    qsort(order, n, sizeof(int), cmp_desc_stable);
    int64_t nk = 0;
    for (int64_t _i = 0; _i < n; _i++) {
        int i = order[_i];
        if (suppressed[i]) continue;
        keep_out[nk++] = i;
        float ix1 = boxes[4 * i + 0], iy1 = boxes[4 * i + 1];
        float ix2 = boxes[4 * i + 2], iy2 = boxes[4 * i + 3];
        float iarea = areas[i];
        for (int64_t _j = _i + 1; _j < n; _j++) {
            int j = order[_j];
            if (suppressed[j]) continue;
            float xx1 = ix1 > boxes[4 * j + 0] ? ix1 : boxes[4 * j + 0];
            float yy1 = iy1 > boxes[4 * j + 1] ? iy1 : boxes[4 * j + 1];
            float xx2 = ix2 < boxes[4 * j + 2] ? ix2 : boxes[4 * j + 2];
            float yy2 = iy2 < boxes[4 * j + 3] ? iy2 : boxes[4 * j + 3];
            float w = xx2 - xx1;
            if (!(w > 0.0f)) w = 0.0f;
            float h = yy2 - yy1;
            if (!(h > 0.0f)) h = 0.0f;
            float inter = w * h;
            float denom = iarea + areas[j];
            denom = denom - inter;
            float ovr = inter / denom;
            if ((double)ovr > iou_threshold) suppressed[j] = 1;
        }
    }
    free(order);
    free(areas);
    free(suppressed);
    return nk;
}

/*
 * input: [B, C, H, W] fp32 (NCHW); rois: [R,5] (batch_idx, x1, y1, x2, y2);
 * output: [R, C, PH, PW].  aligned = False (the MultiScaleRoIAlign default).
 */
void roi_align_ref(const float* input, int64_t B, int64_t C, int64_t H, int64_t W,
                   const float* rois, int64_t R, float spatial_scale, int PH, int PW,
                   int sampling_ratio, float* output) {
    (void)B;
    for (int64_t n = 0; n < R; n++) {
        const float* r = rois + 5 * n;
        int64_t bi = (int64_t)r[0];
        float roi_start_w = r[1] * spatial_scale;
        float roi_start_h = r[2] * spatial_scale;
        float roi_end_w = r[3] * spatial_scale;
        float roi_end_h = r[4] * spatial_scale;
        float roi_width = roi_end_w - roi_start_w;
        float roi_height = roi_end_h - roi_start_h;
        if (roi_width < 1.0f) roi_width = 1.0f;
        if (roi_height < 1.0f) roi_height = 1.0f;
        float bin_h = roi_height / (float)PH;
        float bin_w = roi_width / (float)PW;
        int gh = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(roi_height / PH);
        int gw = sampling_ratio > 0 ? sampling_ratio : (int)ceilf(roi_width / PW);
        int cnt = gh * gw;
        float count = (float)(cnt > 1 ? cnt : 1);
        int npc = PH * PW * gh * gw;
        int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * 4 * npc);
        float* wts = (float*)malloc(sizeof(float) * 4 * npc);
        int pc = 0;
        for (int ph = 0; ph < PH; ph++)
            for (int pw = 0; pw < PW; pw++)
                for (int iy = 0; iy < gh; iy++) {
                    float yy = roi_start_h + (float)ph * bin_h +
                               (float)(iy + .5f) * bin_h / (float)gh;
                    for (int ix = 0; ix < gw; ix++) {
                        float xx = roi_start_w + (float)pw * bin_w +
                                   (float)(ix + .5f) * bin_w / (float)gw;
                        float x = xx, y = yy;
                        if (y < -1.0f || y > (float)H || x < -1.0f || x > (float)W) {
                            for (int q = 0; q < 4; q++) { pos[4 * pc + q] = 0; wts[4 * pc + q] = 0.f; }
                            pc++;
                            continue;
                        }
                        if (y <= 0) y = 0;
                        if (x <= 0) x = 0;
                        int y_low = (int)y, x_low = (int)x, y_high, x_high;
                        if (y_low >= H - 1) { y_high = y_low = (int)H - 1; y = (float)y_low; }
                        else y_high = y_low + 1;
                        if (x_low >= W - 1) { x_high = x_low = (int)W - 1; x = (float)x_low; }
                        else x_high = x_low + 1;
                        float ly = y - y_low, lx = x - x_low;
                        float hy = 1.f - ly, hx = 1.f - lx;
                        pos[4 * pc + 0] = (int64_t)y_low * W + x_low;
                        pos[4 * pc + 1] = (int64_t)y_low * W + x_high;
                        pos[4 * pc + 2] = (int64_t)y_high * W + x_low;
                        pos[4 * pc + 3] = (int64_t)y_high * W + x_high;
                        wts[4 * pc + 0] = hy * hx;
                        wts[4 * pc + 1] = hy * lx;
                        wts[4 * pc + 2] = ly * hx;
                        wts[4 * pc + 3] = ly * lx;
                        pc++;
                    }
                }
        for (int64_t c = 0; c < C; c++) {
            const float* in = input + (bi * C + c) * H * W;
            float* out = output + ((n * C + c) * PH) * PW;
            int p = 0;
            for (int ph = 0; ph < PH; ph++)
                for (int pw = 0; pw < PW; pw++) {
                    float v = 0.f;
                    for (int s = 0; s < gh * gw; s++, p++) {
                        float t0 = wts[4 * p + 0] * in[pos[4 * p + 0]];
                        float t1 = wts[4 * p + 1] * in[pos[4 * p + 1]];
                        float t2 = wts[4 * p + 2] * in[pos[4 * p + 2]];
                        float t3 = wts[4 * p + 3] * in[pos[4 * p + 3]];
                        float t = t0 + t1;
                        t = t + t2;
                        t = t + t3;
                        v += t;
                    }
                    out[ph * PW + pw] = v / count;
                }
        }
        free(pos);
        free(wts);
    }
}
