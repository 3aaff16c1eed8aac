// pybind11 shims for the gfx950 kernels.  Tensors cross the boundary as raw
// device pointers (torch.Tensor.data_ptr()) and the HIP stream as an integer
// (torch.cuda.current_stream().cuda_stream), so this module needs neither torch
// headers nor a JIT: it is built in-tree by govideocompressor_amd/_build.py.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "../common/hevc_ctu_coder.h"
#include "hevc_decode.h"

namespace py = pybind11;

extern "C" {
long long mivc_hevc_entropy_state_bytes(int W, int H);
int mivc_launch_hevc_entropy(const void* pic, int B, const int* qp, const void* ctu, const void* cu, const void* col,
                             const unsigned long long* nzmap, const int16_t* cy, const int16_t* cb, const int16_t* cr,
                             uint8_t* state, long long state_bytes, uint8_t* out, unsigned cap, unsigned* sizes,
                             int* errs, unsigned long long* offs, unsigned long long* offs_host, uint8_t* dst,
                             unsigned long long dst_cap, int* overflow, void* stream, unsigned long long* prof,
                             int* gprog, void* gctx);
int mivc_launch_hevc_decode(const mivc::gpu::HevcDecParams* p, int stage, void* stream);
void mivc_launch_synth(void* y, void* u, void* v, int width, int height, int slots, int frames, int frame0,
                       uint32_t seed, int bit_depth, int slot0, void* stream, int kind);
void mivc_launch_prep(const uint8_t* in_y, const uint8_t* in_u, const uint8_t* in_v, int w, int h,
                      int64_t in_stride_y, int64_t in_stride_c, int nframes, uint8_t* out_y, uint8_t* out_u,
                      uint8_t* out_v, int ow, int oh, int W, int H, void* stream, const int* fsel);
void mivc_launch_rgb_to_i420(const uint8_t* rgb, int w, int h, int nframes, uint8_t* y, uint8_t* u, uint8_t* v,
                             void* stream);
void mivc_launch_me(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref_y, const int16_t* pred_mv,
                    int16_t* out_mv, int* out_cost, uint8_t* out_pred, int* out_intra_cost, const int* qp, int range,
                    int subpel, uint8_t* hp, const int8_t* aq, int planes_ready, int early_sad, void* stream,
                    const int* gate_cost, int gate_thresh, const int16_t* cost_mv, const void* route, int nbuf,
                    int role, int want, const int16_t* seed_mv);
void mivc_launch_me_ref_select(int B, int wmb, int hmb, int nref, int16_t* mv, int16_t* mv8, int* cost, uint8_t* pred,
                               const int16_t* xmv, const int* xcost, const uint8_t* xpred, int8_t* mref, const int* qp,
                               const int8_t* aq, void* stream, const void* route);
void mivc_launch_b_spatial(int B, int wmb, int hmb, void* hdr, const void* col, const uint8_t* src, const uint8_t* ref1,
                           const uint8_t* hp1, const uint8_t* const* ref0k, const uint8_t* const* hp0k, const int* w1,
                           int nref, uint8_t* pred_out, int* err, void* stream, const int* intra_cost, int* cost,
                           const int* qp, const int8_t* aq, int bias, const void* route, int nbuf);
void mivc_launch_b_direct(int B, int wmb, int hmb, const void* col, const int* dsf, const int* direct_copy, int nref,
                          int16_t* dmv, int8_t* dref, int16_t* pm0, int16_t* pm1, void* stream, const void* route,
                          int nbuf, uint8_t* czero);
void mivc_launch_b_spatial_exact(int B, int wmb, int hmb, void* hdr, const int* intra_cost, const int* cost,
                                 const uint8_t* czero, uint8_t* fix, void* stream, const void* route, int slice_rows,
                                 int tol);
void mivc_launch_b_spatial_fixup(int B, int wmb, int hmb, const void* hdr, const uint8_t* fix, const uint8_t* ref0,
                                 const uint8_t* hp0, const uint8_t* ref1, const uint8_t* hp1, uint8_t* pred_out,
                                 void* stream, const void* route, int nbuf);
void mivc_launch_p_refine(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref, const uint8_t* hp,
                          const int16_t* mv_in, int16_t* mv_out, int* cost, const int16_t* pm, uint8_t* pred,
                          const int* qp, const int8_t* aq, void* stream, const void* route, int nbuf,
                          const uint8_t* chg_in, uint8_t* chg_out);
void mivc_launch_b_decide(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref0, const uint8_t* ref1,
                          const uint8_t* hp0, const uint8_t* hp1, const int16_t* mv0, const int16_t* mv1,
                          const int* cost0, const int* cost1, const uint8_t* pred0, const uint8_t* pred1,
                          const int16_t* pm0, const int16_t* pm1, const int16_t* dmv, const int* qp, const int8_t* aq,
                          void* hdr, uint8_t* pred_out, int* cost_out, void* stream, const int* w1, int nref,
                          const int8_t* dref, const uint8_t* const* ref0k, const uint8_t* const* hp0k,
                          int direct_only, int bparts, int have_direct, int spatial, int dbias, const void* route,
                          int nbuf, const uint8_t* czero);
void mivc_launch_aq_offsets(int B, int wmb, int hmb, const uint8_t* sy, const uint8_t* su, const uint8_t* sv,
                            float strength, const float* extra, long long extra_stride, int8_t* out, void* stream,
                            const void* route);
void mivc_launch_mbtree(int B, int F, int lbw, int lbh, const int* blk_cost, const int* blk_mv, void* prop,
                        float strength, float* out, void* stream);
void mivc_launch_qp_fixup(int B, int wmb, int hmb, void* hdr, const int16_t* coef, const uint8_t* nz, uint8_t* flags,
                          const int* slice_qp, void* stream, int slice_rows);
void mivc_launch_me_halfpel(int B, int W, int H, const uint8_t* ref_y, uint8_t* hp, void* stream, const void* route,
                            int nbuf);
void mivc_launch_encode_inter(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* src_u,
                              const uint8_t* src_v, const uint8_t* ref_y, const uint8_t* ref_u, const uint8_t* ref_v,
                              uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v, const uint8_t* pred_y,
                              const int16_t* mv, const int* me_cost, const int* intra_cost, const int* qp,
                              int chroma_qp_offset, void* hdr, int16_t* coef, uint8_t* nz, uint8_t* intra_flag,
                              int* intra_count, const int8_t* aq, const uint8_t* ref1_u, const uint8_t* ref1_v,
                              int bmode, int t8, const int16_t* mv8, void* stream, const int* w1, int nref,
                              const uint8_t* const* xref_u, const uint8_t* const* xref_v, const int8_t* mref,
                              const int* wp, int trellis, float trellis_lambda, const void* route, int nbuf);
void mivc_launch_wp_stats16(const uint16_t* y, const uint16_t* u, const uint16_t* v, int w, int h, int npics,
                            unsigned long long* out, void* stream);
void mivc_launch_wp_stats(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h, int npics,
                          unsigned long long* out, void* stream);
void mivc_launch_wp_src(const uint8_t* src, uint8_t* dst, const int* wt, int B, long long plane_bytes, void* stream);
void mivc_launch_p_part8(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref, const uint8_t* hp,
                         const int16_t* mv, const int16_t* pm, int* cost, uint8_t* pred, int16_t* mv8, const int* qp,
                         const int8_t* aq, int overhead, int min_satd, void* stream, const void* route, int nbuf,
                         const int* bits16, const uint8_t* dir16);
void mivc_launch_encode_intra(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* src_u,
                              const uint8_t* src_v, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v, const int* qp,
                              int chroma_qp_offset, void* hdr, int16_t* coef, uint8_t* nz,
                              const uint8_t* intra_flag, const int* intra_count, int* err, int use_i4x4,
                              const int8_t* aq, void* stream, int use_i8x8, const void* route, int nbuf,
                              int slice_rows, int trellis, float trellis_lambda, int* gprog, long long gprog_ints);
void mivc_launch_deblock(int B, int wmb, int hmb, uint8_t* rec_y, uint8_t* rec_u, uint8_t* rec_v, const void* hdr,
                         const uint8_t* nz, int chroma_qp_offset, int alpha_off, int beta_off, int* err,
                         void* stream, const void* route, int nbuf);
void mivc_launch_decode_picture_dpb(int B, int wmb, int hmb, int dpb_n, uint8_t* dpb_y, uint8_t* dpb_u, uint8_t* dpb_v,
                                    const int16_t* cur_idx, const int16_t* reftab, const int16_t* wp, const int16_t* sub,
                                    const void* hdr, const uint32_t* mask, const uint32_t* off,
                                    const int16_t* coef, const int8_t* run, int any_inter, int chroma_qp_offset,
                                    uint8_t* nz, int* err, void* stream);
void mivc_launch_deblock_dpb(int B, int wmb, int hmb, int dpb_n, uint8_t* dpb_y, uint8_t* dpb_u, uint8_t* dpb_v,
                             const int16_t* cur_idx, const void* hdr, const uint8_t* nz, const uint8_t* bs,
                             int chroma_qp_offset, int alpha_off, int beta_off, int* err, void* stream);
int mivc_launch_scale(const void* in, int w, int h, long long in_stride, long long in_pitch, void* out, int ow, int oh,
                      int W, int H, long long out_stride, long long out_pitch, int nframes, const int* fx,
                      const int16_t* cx, int tx, const int* fy, const int16_t* cy, int ty, int tile_w, int tile_h,
                      int in_cols, int in_rows, int bd, void* stream);
void mivc_launch_hevc_intra(int B, int W, int H, const uint16_t* sy, const uint16_t* su, const uint16_t* sv,
                            uint16_t* ry, uint16_t* ru, uint16_t* rv, void* ctu, void* cu, int16_t* cy, int16_t* cu_,
                            int16_t* cv, const int* qp, const int8_t* run, int* cand, int bd, int analyze, int recon,
                            int* err, int sdh, const uint8_t* ctb_mask, void* stream, int ctu64);
void mivc_launch_hevc_inter(int B, int W, int H, const uint16_t* sy, const uint16_t* su, const uint16_t* sv,
                            const uint16_t* fy, const uint16_t* fu, const uint16_t* fv, uint16_t* ry, uint16_t* ru,
                            uint16_t* rv, void* ctu, void* cu, int16_t* cy, int16_t* cu_, int16_t* cv, const int* qp,
                            const int8_t* run, const int* cand, const int16_t* mv, const int* me_cost, int bd,
                            int tu_split, int sdh, int intra_bias, void* stream, const int16_t* mvb,
                            const uint8_t* dirb, const uint16_t* f1y, const uint16_t* f1u, const uint16_t* f1v,
                            const int16_t* wp, const uint16_t* const* xref, const int16_t* mv8);
void mivc_launch_hevc_b(int mode, int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref0, const uint8_t* ref1,
                        const uint8_t* hp0, const uint8_t* hp1, const int16_t* mv0, const int16_t* mv1, const int* cost0,
                        const int* cost1, const int16_t* pm0, const int16_t* pm1, const int16_t* tmv, const uint8_t* tdir,
                        const int16_t* mvb_in, const uint8_t* dir_in, int16_t* mvb_out, uint8_t* dir_out, int* cost,
                        int* bits, const int* qp, const int8_t* aq, void* stream, int bslice, int max_merge, int ctu64, const uint8_t* chg_in, uint8_t* chg_out,
                        int nref0, const uint8_t* const* xref, const uint8_t* const* xhp, const int16_t* xmv,
                        const int* xcost, const int16_t* xpm);
void mivc_launch_hevc_deblock(int B, int W, int H, int bd, uint16_t* y, uint16_t* u, uint16_t* v, const void* cu,
                              const void* ctu, const int8_t* run, void* stream);
void mivc_launch_hevc_aq(int B, int W, int H, int bd, const uint16_t* sy, const uint16_t* su, const uint16_t* sv,
                         const int* qp, float strength, const float* extra, long long extra_stride, int extra_rows,
                         int* ctb_qp, int8_t* mb_aq, void* stream);
void mivc_launch_hevc_pack_levels(int B, int W, int H, const int16_t* cy, const int16_t* cb, const int16_t* cr,
                                  unsigned long long* nzmap, int* cnt, unsigned* off, long long cap_blocks, int16_t* out,
                                  int* err, void* stream);
void mivc_launch_hevc_merge_refine(int B, int wmb, int hmb, const uint8_t* src_y, const uint8_t* ref, const uint8_t* hp,
                                   const int16_t* mv_in, int16_t* mv_out, int* cost, const int16_t* pm, const int* qp,
                                   const int8_t* aq, void* stream);
void mivc_launch_hevc_qp_fixup(int B, int W, int H, void* ctu, const void* cu, const int* qp, const int8_t* run,
                               int wpp, void* stream, int ctu64);
void mivc_launch_hevc_sao(int B, int W, int H, int bd, const uint16_t* dy, const uint16_t* du, const uint16_t* dv,
                          uint16_t* y, uint16_t* u, uint16_t* v, const uint16_t* sy, const uint16_t* su,
                          const uint16_t* sv, void* ctu, const int* qp, const int8_t* run, int enable, void* stream, int ctu64);
size_t mivc_cavlc_mb_bytes();
size_t mivc_cabac_nb_bytes();
int mivc_cabac_gap();
void mivc_launch_cabac_bin(int B, int wmb, int hmb, const void* hdr, const int16_t* coef, uint32_t* mask, void* nb,
                           int* cnt, long long* off, int* tot, uint16_t* pool, long long pool_cap,
                           long long* pool_used, long long* base, int* total, const int* slot_qp, int slice_type,
                           int num_ref_l0, int num_ref_l1, int t8x8_mode, int* err, void* stream, const void* route,
                           int slice_rows);
void mivc_launch_cabac_code(int L, int B, uint16_t* pool, const long long* base, const int* total,
                            const uint32_t* hdr_bits, const int* hdr_nbits, const int* slot_qp,
                            unsigned long long itypes, int* bytes, uint8_t* out, long long* out_off, int* err,
                            uint8_t* host_out, long long host_cap, void* stream);
void mivc_launch_cavlc(int B, int wmb, int hmb, const void* hdr, const int16_t* coef, void* mbs, int* len,
                       long long* off, int* trail, long long* total_bits, int* slot_bytes, uint32_t* words,
                       long long cap_words, const uint32_t* hdr_bits, const int* hdr_nbits, int pslice, int slice_qp,
                       const int* slot_qp, uint8_t* out, long long* out_off, const uint8_t* nz, void* stream);
void mivc_launch_satd_blocks(const uint8_t* src, const uint8_t* pred, int* out, int n, int mode, void* stream);
void mivc_launch_trellis_blocks(const int* w, int* out, int n, int qp, int mode, int skip_dc, void* stream);
void mivc_launch_sse(int B, int W, int H, int w, int h, const uint8_t* sy, const uint8_t* su, const uint8_t* sv,
                     const uint8_t* ry, const uint8_t* ru, const uint8_t* rv, unsigned long long* sse,
                     float* ssim_sum, void* stream, const void* route, int nbuf);
long long mivc_lookahead_low_bytes(int w, int h, int N);
int mivc_launch_lookahead_multi(const uint8_t* low, int w, int h, int N, int F, const int* blk_cost, const int* blk_mv,
                                int D, int range, unsigned long long* out, void* stream, const float* wt);
int mivc_launch_hevc_prep_frame(int B, const void* sy, const void* su, const void* sv, long long ss_y, long long ss_c,
                                int pitch_y, int pitch_c, int bps, int w, int h, uint16_t* dy, uint16_t* du,
                                uint16_t* dv, uint8_t* d8, int W, int H, int shift, int bd, void* stream);
int mivc_launch_hevc_proxy8(const uint16_t* src, uint8_t* dst, long long n, int shift, void* stream);
int mivc_launch_lookahead(const uint8_t* y, int w, int h, long long fstride, int N, int F, uint8_t* low,
                          unsigned long long* frame_cost, int* blk_cost, int* blk_mv, int range, void* stream,
                          uint8_t* low4, int* mv4, unsigned long long* cost4, float* wt, unsigned long long* wstats,
                          float thr_mean, float thr_scale, int stage);
long long mivc_lookahead_quarter_bytes(int w, int h, int N);
}

namespace {
template <class T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
void* S(uintptr_t s) { return reinterpret_cast<void*>(s); }
}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "govideocompressor_amd gfx950 kernels (raw-pointer launch shims)";
  m.attr("arch") = "gfx950";

  m.def("synth", [](uintptr_t y, uintptr_t u, uintptr_t v, int w, int h, int slots, int frames, int frame0,
                    uint32_t seed, uintptr_t stream, int bit_depth, int slot0, int kind) {
    if (bit_depth != 8 && bit_depth != 10) throw std::invalid_argument("synth: bit_depth must be 8 or 10");
    if (kind < 0 || kind > 6) throw std::invalid_argument("synth: content kind 0..6");
    mivc_launch_synth(P<void>(y), P<void>(u), P<void>(v), w, h, slots, frames, frame0, seed, bit_depth, slot0,
                      S(stream), kind);
  }, py::arg("y"), py::arg("u"), py::arg("v"), py::arg("w"), py::arg("h"), py::arg("slots"), py::arg("frames"),
     py::arg("frame0"), py::arg("seed"), py::arg("stream"), py::arg("bit_depth") = 8, py::arg("slot0") = 0,
     py::arg("kind") = 0);
  m.def("prep", [](uintptr_t iy, uintptr_t iu, uintptr_t iv, int w, int h, int64_t sy, int64_t sc, int n,
                   uintptr_t oy, uintptr_t ou, uintptr_t ov, int ow, int oh, int W, int H, uintptr_t stream,
                   uintptr_t fsel) {
    // fsel (nullable): int32 [n] frame index per input slot, added to the slot's frame 0
    if (ow != w || oh != h) throw std::invalid_argument("prep: resample with ops.scale (scale.hip) first");
    if (W < w || H < h || w < 2 || h < 2) throw std::invalid_argument("prep: bad geometry");
    mivc_launch_prep(P<uint8_t>(iy), P<uint8_t>(iu), P<uint8_t>(iv), w, h, sy, sc, n, P<uint8_t>(oy), P<uint8_t>(ou),
                     P<uint8_t>(ov), ow, oh, W, H, S(stream), P<int>(fsel));
  }, py::arg("iy"), py::arg("iu"), py::arg("iv"), py::arg("w"), py::arg("h"), py::arg("sy"), py::arg("sc"), py::arg("n"),
     py::arg("oy"), py::arg("ou"), py::arg("ov"), py::arg("ow"), py::arg("oh"), py::arg("W"), py::arg("H"),
     py::arg("stream"), py::arg("fsel") = 0);
  m.def("rgb_to_i420", [](uintptr_t rgb, int w, int h, int n, uintptr_t y, uintptr_t u, uintptr_t v,
                          uintptr_t stream) {
    mivc_launch_rgb_to_i420(P<uint8_t>(rgb), w, h, n, P<uint8_t>(y), P<uint8_t>(u), P<uint8_t>(v), S(stream));
  });
  m.def("me", [](int B, int wmb, int hmb, uintptr_t src, uintptr_t ref, uintptr_t pred_mv, uintptr_t out_mv,
                 uintptr_t out_cost, uintptr_t out_pred, uintptr_t out_intra, uintptr_t qp, int range, int subpel,
                 uintptr_t stream, uintptr_t hp, uintptr_t aq, int planes_ready, int early_sad, uintptr_t gate_cost,
                 int gate_thresh, uintptr_t cost_mv, uintptr_t route, int nbuf, int role, int want, uintptr_t seed_mv) {
    if (planes_ready && !hp) throw std::invalid_argument("me: planes_ready needs the hp buffer");
    if (route && (nbuf < 1 || role < 0 || role > 4 || (want != 0 && want != 1) || !planes_ready))
      throw std::invalid_argument("me: a routed search needs nbuf, a role (list-0 0..3 / list-1 4), want P/B and the planes");
    mivc_launch_me(B, wmb, hmb, P<uint8_t>(src), P<uint8_t>(ref), P<int16_t>(pred_mv), P<int16_t>(out_mv),
                   P<int>(out_cost), P<uint8_t>(out_pred), P<int>(out_intra), P<int>(qp), range, subpel,
                   P<uint8_t>(hp), P<int8_t>(aq), planes_ready, early_sad, S(stream), P<int>(gate_cost), gate_thresh,
                   P<int16_t>(cost_mv), P<void>(route), nbuf, role, want, P<int16_t>(seed_mv));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("src"), py::arg("ref"), py::arg("pred_mv"),
     py::arg("out_mv"), py::arg("out_cost"), py::arg("out_pred"), py::arg("out_intra"), py::arg("qp"),
     py::arg("range"), py::arg("subpel"), py::arg("stream"), py::arg("hp") = 0, py::arg("aq") = 0,
     py::arg("planes_ready") = 0, py::arg("early_sad") = 0, py::arg("gate_cost") = 0, py::arg("gate_thresh") = 0,
     py::arg("cost_mv") = 0, py::arg("route") = 0, py::arg("nbuf") = 0, py::arg("role") = 0, py::arg("want") = 0,
     py::arg("seed_mv") = 0);
  m.def("me_ref_select", [](int B, int wmb, int hmb, int nref, uintptr_t mv, uintptr_t mv8, uintptr_t cost,
                            uintptr_t pred, uintptr_t xmv, uintptr_t xcost, uintptr_t xpred, uintptr_t mref,
                            uintptr_t qp, uintptr_t aq, uintptr_t stream, uintptr_t route) {
    if (nref < 2 || nref > 4) throw std::invalid_argument("me_ref_select: nref in 2..4");
    mivc_launch_me_ref_select(B, wmb, hmb, nref, P<int16_t>(mv), P<int16_t>(mv8), P<int>(cost), P<uint8_t>(pred),
                              P<int16_t>(xmv), P<int>(xcost), P<uint8_t>(xpred), P<int8_t>(mref), P<int>(qp),
                              P<int8_t>(aq), S(stream), P<void>(route));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("nref"), py::arg("mv"), py::arg("mv8"), py::arg("cost"),
     py::arg("pred"), py::arg("xmv"), py::arg("xcost"), py::arg("xpred"), py::arg("mref"), py::arg("qp"), py::arg("aq"),
     py::arg("stream"), py::arg("route") = 0);
  m.def("b_spatial", [](int B, int wmb, int hmb, uintptr_t hdr, uintptr_t col, uintptr_t src, uintptr_t ref1,
                        uintptr_t hp1, std::vector<uintptr_t> ref0k, std::vector<uintptr_t> hp0k, std::vector<int> w1,
                        uintptr_t pred_out, uintptr_t err, uintptr_t stream, uintptr_t intra_cost, uintptr_t cost,
                        uintptr_t qp, uintptr_t aq, int bias, uintptr_t route, int nbuf) {
    // spatial direct: exact derivation + direct-vs-explicit decision in MB wavefront order;
    // ref0k / hp0k / w1: every list-0 picture (entry 0 = RefPicList0[0]); routed: the pools
    const size_t n = ref0k.size();
    if (n < 1 || n > 4 || hp0k.size() != n || w1.size() != n)
      throw std::invalid_argument("b_spatial: 1..4 list-0 pictures with planes and weights");
    if (hmb > 272 || wmb > 480) throw std::invalid_argument("b_spatial: at most 272 MB rows and 480 columns");
    const uint8_t* rk[4];
    const uint8_t* hk[4];
    for (size_t i = 0; i < n; ++i) {
      rk[i] = P<uint8_t>(ref0k[i]);
      hk[i] = P<uint8_t>(hp0k[i]);
    }
    mivc_launch_b_spatial(B, wmb, hmb, P<void>(hdr), P<void>(col), P<uint8_t>(src), P<uint8_t>(ref1), P<uint8_t>(hp1),
                          rk, hk, w1.data(), static_cast<int>(n), P<uint8_t>(pred_out), P<int>(err), S(stream),
                          P<int>(intra_cost), P<int>(cost), P<int>(qp), P<int8_t>(aq), bias, P<void>(route), nbuf);
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("hdr"), py::arg("col"), py::arg("src"), py::arg("ref1"),
     py::arg("hp1"), py::arg("ref0k"), py::arg("hp0k"), py::arg("w1"), py::arg("pred_out"), py::arg("err"),
     py::arg("stream"), py::arg("intra_cost"), py::arg("cost"), py::arg("qp"), py::arg("aq"), py::arg("bias"),
     py::arg("route") = 0, py::arg("nbuf") = 0);
  m.def("b_direct", [](int B, int wmb, int hmb, uintptr_t col, std::vector<int> dsf, std::vector<int> direct_copy,
                       uintptr_t dmv, uintptr_t pm0, uintptr_t pm1, uintptr_t stream, uintptr_t dref, uintptr_t route,
                       int nbuf, uintptr_t czero) {
    if (dsf.empty() || dsf.size() > 4 || dsf.size() != direct_copy.size())
      throw std::invalid_argument("b_direct: one (dsf, direct_copy) pair per list-0 picture, at most 4");
    if (route && nbuf < 1) throw std::invalid_argument("b_direct: a routed launch needs the pool size");
    mivc_launch_b_direct(B, wmb, hmb, P<void>(col), dsf.data(), direct_copy.data(), static_cast<int>(dsf.size()),
                         P<int16_t>(dmv), P<int8_t>(dref), P<int16_t>(pm0), P<int16_t>(pm1), S(stream), P<void>(route),
                         nbuf, P<uint8_t>(czero));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("col"), py::arg("dsf"), py::arg("direct_copy"),
     py::arg("dmv"), py::arg("pm0"), py::arg("pm1"), py::arg("stream"), py::arg("dref") = 0, py::arg("route") = 0,
     py::arg("nbuf") = 0, py::arg("czero") = 0);
  m.def("b_spatial_exact", [](int B, int wmb, int hmb, uintptr_t hdr, uintptr_t intra_cost, uintptr_t cost,
                              uintptr_t czero, uintptr_t fix, uintptr_t stream, uintptr_t route, int slice_rows,
                              int tol) {
    // spatial direct, fast path: the exact direct motion in decoding order (one lane per MB row)
    if (hmb > 320 || wmb > 480) throw std::invalid_argument("b_spatial_exact: at most 320 MB rows and 480 columns");
    if (!hdr || !intra_cost || !cost || !czero || !fix) throw std::invalid_argument("b_spatial_exact: null buffer");
    mivc_launch_b_spatial_exact(B, wmb, hmb, P<void>(hdr), P<int>(intra_cost), P<int>(cost), P<uint8_t>(czero),
                                P<uint8_t>(fix), S(stream), P<void>(route), slice_rows, tol);
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("hdr"), py::arg("intra_cost"), py::arg("cost"),
     py::arg("czero"), py::arg("fix"), py::arg("stream"), py::arg("route") = 0, py::arg("slice_rows") = 0,
     py::arg("tol") = -1);
  m.def("b_spatial_fixup", [](int B, int wmb, int hmb, uintptr_t hdr, uintptr_t fix, uintptr_t ref0, uintptr_t hp0,
                              uintptr_t ref1, uintptr_t hp1, uintptr_t pred_out, uintptr_t stream, uintptr_t route,
                              int nbuf) {
    if (!route || nbuf < 1) throw std::invalid_argument("b_spatial_fixup: routed launches only");
    mivc_launch_b_spatial_fixup(B, wmb, hmb, P<void>(hdr), P<uint8_t>(fix), P<uint8_t>(ref0), P<uint8_t>(hp0),
                                P<uint8_t>(ref1), P<uint8_t>(hp1), P<uint8_t>(pred_out), S(stream), P<void>(route),
                                nbuf);
  });
  m.def("p_refine", [](int B, int wmb, int hmb, uintptr_t src, uintptr_t ref, uintptr_t hp, uintptr_t mv_in,
                       uintptr_t mv_out, uintptr_t cost, uintptr_t pm, uintptr_t pred, uintptr_t qp, uintptr_t aq,
                       uintptr_t stream, uintptr_t route, int nbuf, uintptr_t chg_in, uintptr_t chg_out) {
    if (mv_in == mv_out) throw std::invalid_argument("p_refine: mv_in and mv_out must differ (Jacobi pass)");
    if (chg_in && chg_in == chg_out) throw std::invalid_argument("p_refine: chg_in and chg_out must differ");
    mivc_launch_p_refine(B, wmb, hmb, P<uint8_t>(src), P<uint8_t>(ref), P<uint8_t>(hp), P<int16_t>(mv_in),
                         P<int16_t>(mv_out), P<int>(cost), P<int16_t>(pm), P<uint8_t>(pred), P<int>(qp),
                         P<int8_t>(aq), S(stream), P<void>(route), nbuf, P<uint8_t>(chg_in), P<uint8_t>(chg_out));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("src"), py::arg("ref"), py::arg("hp"), py::arg("mv_in"),
     py::arg("mv_out"), py::arg("cost"), py::arg("pm"), py::arg("pred"), py::arg("qp"), py::arg("aq"),
     py::arg("stream"), py::arg("route") = 0, py::arg("nbuf") = 0, py::arg("chg_in") = 0, py::arg("chg_out") = 0);
  m.def("b_decide", [](int B, int wmb, int hmb, uintptr_t src, uintptr_t ref0, uintptr_t ref1, uintptr_t hp0,
                       uintptr_t hp1, uintptr_t mv0, uintptr_t mv1, uintptr_t cost0, uintptr_t cost1, uintptr_t pred0,
                       uintptr_t pred1, uintptr_t pm0, uintptr_t pm1, uintptr_t dmv, uintptr_t qp, uintptr_t aq,
                       uintptr_t hdr, uintptr_t pred_out, uintptr_t cost_out, uintptr_t stream, std::vector<int> w1,
                       uintptr_t dref, std::vector<uintptr_t> ref0k, std::vector<uintptr_t> hp0k, int direct_only, int bparts, int have_direct,
                       int spatial, int dbias, uintptr_t route, int nbuf, uintptr_t czero) {
    // w1: implicit list-1 weight per list-0 picture; ref0k / hp0k: luma / half-sample planes of
    // RefPicList0[1..] (direct prediction of quadrants whose co-located block used a farther picture)
    if (w1.empty() || w1.size() > 4) throw std::invalid_argument("b_decide: one implicit weight per list-0 picture");
    for (int v : w1)
      if (v < -64 || v > 128) throw std::invalid_argument("b_decide: implicit weight w1 in -64..128");
    const size_t n = w1.size();
    if (n > 1 && (ref0k.size() != n - 1 || hp0k.size() != n - 1 || !dref))
      throw std::invalid_argument("b_decide: several list-0 pictures need their planes and the direct refIdx");
    const uint8_t* rk[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint8_t* hk[4] = {nullptr, nullptr, nullptr, nullptr};
    for (size_t i = 1; i < n; ++i) {
      rk[i] = P<uint8_t>(ref0k[i - 1]);
      hk[i] = P<uint8_t>(hp0k[i - 1]);
    }
    mivc_launch_b_decide(B, wmb, hmb, P<uint8_t>(src), P<uint8_t>(ref0), P<uint8_t>(ref1), P<uint8_t>(hp0),
                         P<uint8_t>(hp1), P<int16_t>(mv0), P<int16_t>(mv1), P<int>(cost0), P<int>(cost1),
                         P<uint8_t>(pred0), P<uint8_t>(pred1), P<int16_t>(pm0), P<int16_t>(pm1), P<int16_t>(dmv),
                         P<int>(qp), P<int8_t>(aq), P<void>(hdr), P<uint8_t>(pred_out), P<int>(cost_out), S(stream),
                         w1.data(), static_cast<int>(n), (n > 1 || route) ? P<int8_t>(dref) : nullptr, rk, hk, direct_only,
                         bparts, have_direct, spatial, dbias, P<void>(route), nbuf, P<uint8_t>(czero));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("src"), py::arg("ref0"), py::arg("ref1"), py::arg("hp0"),
     py::arg("hp1"), py::arg("mv0"), py::arg("mv1"), py::arg("cost0"), py::arg("cost1"), py::arg("pred0"),
     py::arg("pred1"), py::arg("pm0"), py::arg("pm1"), py::arg("dmv"), py::arg("qp"), py::arg("aq"), py::arg("hdr"),
     py::arg("pred_out"), py::arg("cost_out"), py::arg("stream"), py::arg("w1") = std::vector<int>{32},
     py::arg("dref") = 0, py::arg("ref0k") = std::vector<uintptr_t>{}, py::arg("hp0k") = std::vector<uintptr_t>{},
     py::arg("direct_only") = 0, py::arg("bparts") = 0, py::arg("have_direct") = 0, py::arg("spatial") = 0, py::arg("dbias") = 0,
     py::arg("route") = 0, py::arg("nbuf") = 0, py::arg("czero") = 0);
  m.def("aq_offsets", [](int B, int wmb, int hmb, uintptr_t sy, uintptr_t su, uintptr_t sv, float strength,
                         uintptr_t out, uintptr_t stream, uintptr_t extra, long long extra_stride, uintptr_t route) {
    mivc_launch_aq_offsets(B, wmb, hmb, P<uint8_t>(sy), P<uint8_t>(su), P<uint8_t>(sv), strength, P<float>(extra),
                           extra_stride, P<int8_t>(out), S(stream), P<void>(route));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("sy"), py::arg("su"), py::arg("sv"), py::arg("strength"),
     py::arg("out"), py::arg("stream"), py::arg("extra") = 0, py::arg("extra_stride") = 0, py::arg("route") = 0);
  m.def("mbtree", [](int B, int F, int lbw, int lbh, uintptr_t blk_cost, uintptr_t blk_mv, uintptr_t prop,
                     float strength, uintptr_t out, uintptr_t stream) {
    mivc_launch_mbtree(B, F, lbw, lbh, P<int>(blk_cost), P<int>(blk_mv), P<void>(prop), strength, P<float>(out),
                       S(stream));
  });
  m.def("qp_fixup", [](int B, int wmb, int hmb, uintptr_t hdr, uintptr_t coef, uintptr_t nz, uintptr_t flags,
                       uintptr_t slice_qp, uintptr_t stream, int slice_rows) {
    mivc_launch_qp_fixup(B, wmb, hmb, P<void>(hdr), P<int16_t>(coef), P<uint8_t>(nz), P<uint8_t>(flags),
                         P<int>(slice_qp), S(stream), slice_rows);
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("hdr"), py::arg("coef"), py::arg("nz"), py::arg("flags"),
     py::arg("slice_qp"), py::arg("stream"), py::arg("slice_rows") = 0);
  m.def("me_halfpel", [](int B, int W, int H, uintptr_t ref, uintptr_t hp, uintptr_t stream, uintptr_t route, int nbuf) {
    if (route && nbuf < 1) throw std::invalid_argument("me_halfpel: a routed launch needs the pool size");
    mivc_launch_me_halfpel(B, W, H, P<uint8_t>(ref), P<uint8_t>(hp), S(stream), P<void>(route), nbuf);
  }, py::arg("B"), py::arg("W"), py::arg("H"), py::arg("ref"), py::arg("hp"), py::arg("stream"), py::arg("route") = 0,
     py::arg("nbuf") = 0);
  m.def("encode_inter",
        [](int B, int wmb, int hmb, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t fy, uintptr_t fu,
           uintptr_t fv, uintptr_t ry, uintptr_t ru, uintptr_t rv, uintptr_t pred, uintptr_t mv, uintptr_t me_cost,
           uintptr_t intra_cost, uintptr_t qp, int cqo, uintptr_t hdr, uintptr_t coef, uintptr_t nz,
           uintptr_t intra_flag, uintptr_t intra_count, uintptr_t stream, uintptr_t aq, uintptr_t ref1_u,
           uintptr_t ref1_v, int bmode, int t8, uintptr_t mv8, std::vector<int> w1, std::vector<uintptr_t> xref_u,
           std::vector<uintptr_t> xref_v, uintptr_t mref, uintptr_t wp, int trellis, float trellis_lambda,
           uintptr_t route, int nbuf) {
          // xref_u / xref_v: chroma of RefPicList0[1..]; w1: implicit list-1 weight per list-0 picture
          if (bmode && (!ref1_u || !ref1_v)) throw std::invalid_argument("encode_inter: B mode needs the list-1 chroma");
          const size_t n = xref_u.size() + 1;
          if (n > 4 || xref_v.size() != xref_u.size()) throw std::invalid_argument("encode_inter: at most 4 list-0 pictures");
          if ((n > 1 || route) && !bmode && !mref)
            throw std::invalid_argument("encode_inter: P pictures with several references need mref");
          if (route && (nbuf < 1 || n > 1)) throw std::invalid_argument("encode_inter: routed launches take pools");
          std::vector<int> w(n, w1.empty() ? 32 : w1[0]);
          for (size_t i = 0; i < n && i < w1.size(); ++i) w[i] = w1[i];
          const uint8_t* xu[4] = {nullptr, nullptr, nullptr, nullptr};
          const uint8_t* xv[4] = {nullptr, nullptr, nullptr, nullptr};
          for (size_t i = 1; i < n; ++i) {
            xu[i] = P<uint8_t>(xref_u[i - 1]);
            xv[i] = P<uint8_t>(xref_v[i - 1]);
          }
          mivc_launch_encode_inter(B, wmb, hmb, P<uint8_t>(sy), P<uint8_t>(su), P<uint8_t>(sv), P<uint8_t>(fy),
                                   P<uint8_t>(fu), P<uint8_t>(fv), P<uint8_t>(ry), P<uint8_t>(ru), P<uint8_t>(rv),
                                   P<uint8_t>(pred), P<int16_t>(mv), P<int>(me_cost), P<int>(intra_cost), P<int>(qp),
                                   cqo, P<void>(hdr), P<int16_t>(coef), P<uint8_t>(nz), P<uint8_t>(intra_flag),
                                   P<int>(intra_count), P<int8_t>(aq), P<uint8_t>(ref1_u), P<uint8_t>(ref1_v), bmode,
                                   t8, P<int16_t>(mv8), S(stream), w.data(), static_cast<int>(n), xu, xv,
                                   bmode ? nullptr : P<int8_t>(mref), P<int>(wp), trellis, trellis_lambda, P<void>(route),
                                   nbuf);
        }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("sy"), py::arg("su"), py::arg("sv"), py::arg("fy"),
        py::arg("fu"), py::arg("fv"), py::arg("ry"), py::arg("ru"), py::arg("rv"), py::arg("pred"), py::arg("mv"),
        py::arg("me_cost"), py::arg("intra_cost"), py::arg("qp"), py::arg("cqo"), py::arg("hdr"), py::arg("coef"),
        py::arg("nz"), py::arg("intra_flag"), py::arg("intra_count"), py::arg("stream"), py::arg("aq") = 0,
        py::arg("ref1_u") = 0, py::arg("ref1_v") = 0, py::arg("bmode") = 0, py::arg("t8") = 0, py::arg("mv8") = 0,
        py::arg("w1") = std::vector<int>{32}, py::arg("xref_u") = std::vector<uintptr_t>{},
        py::arg("xref_v") = std::vector<uintptr_t>{}, py::arg("mref") = 0, py::arg("wp") = 0, py::arg("trellis") = 0,
        py::arg("trellis_lambda") = 1.0f, py::arg("route") = 0, py::arg("nbuf") = 0);
  m.def("wp_stats16", [](uintptr_t y, uintptr_t u, uintptr_t v, int w, int h, int npics, uintptr_t out, uintptr_t stream) {
    if (w % 2 || h % 2 || npics <= 0) throw std::invalid_argument("wp_stats16: even picture sizes, npics > 0");
    mivc_launch_wp_stats16(P<uint16_t>(y), P<uint16_t>(u), P<uint16_t>(v), w, h, npics, P<unsigned long long>(out),
                           S(stream));
  });
  m.def("wp_stats", [](uintptr_t y, uintptr_t u, uintptr_t v, int w, int h, int npics, uintptr_t out, uintptr_t stream) {
    if (w % 2 || h % 2 || (w * h) % 4) throw std::invalid_argument("wp_stats: even picture sizes");
    mivc_launch_wp_stats(P<uint8_t>(y), P<uint8_t>(u), P<uint8_t>(v), w, h, npics, P<unsigned long long>(out),
                         S(stream));
  });
  m.def("wp_src", [](uintptr_t src, uintptr_t dst, uintptr_t wt, int B, long long plane_bytes, uintptr_t stream) {
    if (plane_bytes % 4) throw std::invalid_argument("wp_src: plane size must be a multiple of 4");
    mivc_launch_wp_src(P<uint8_t>(src), P<uint8_t>(dst), P<int>(wt), B, plane_bytes, S(stream));
  });
  m.def("p_part8", [](int B, int wmb, int hmb, uintptr_t src, uintptr_t ref, uintptr_t hp, uintptr_t mv, uintptr_t pm,
                      uintptr_t cost, uintptr_t pred, uintptr_t mv8, uintptr_t qp, uintptr_t aq, int overhead,
                      int min_satd, uintptr_t stream, uintptr_t route, int nbuf, uintptr_t bits16, uintptr_t dir16) {
    if (!hp || !mv8) throw std::invalid_argument("p_part8: needs the half-sample planes and an mv8 buffer");
    if (!pred && !bits16) throw std::invalid_argument("p_part8: the H.264 form rewrites pred");
    mivc_launch_p_part8(B, wmb, hmb, P<uint8_t>(src), P<uint8_t>(ref), P<uint8_t>(hp), P<int16_t>(mv), P<int16_t>(pm),
                        P<int>(cost), P<uint8_t>(pred), P<int16_t>(mv8), P<int>(qp), P<int8_t>(aq), overhead, min_satd,
                        S(stream), P<void>(route), nbuf, P<int>(bits16), P<uint8_t>(dir16));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("src"), py::arg("ref"), py::arg("hp"), py::arg("mv"),
     py::arg("pm"), py::arg("cost"), py::arg("pred"), py::arg("mv8"), py::arg("qp"), py::arg("aq"), py::arg("overhead"),
     py::arg("min_satd"), py::arg("stream"), py::arg("route") = 0, py::arg("nbuf") = 0, py::arg("bits16") = 0,
     py::arg("dir16") = 0);
  m.def("encode_intra", [](int B, int wmb, int hmb, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t ry,
                           uintptr_t ru, uintptr_t rv, uintptr_t qp, int cqo, uintptr_t hdr, uintptr_t coef,
                           uintptr_t nz, uintptr_t intra_flag, uintptr_t intra_count, uintptr_t err, int use_i4x4,
                           uintptr_t stream, uintptr_t aq, int use_i8x8, uintptr_t route, int nbuf, int slice_rows,
                           int trellis, float trellis_lambda, uintptr_t gprog, long long gprog_ints) {
    mivc_launch_encode_intra(B, wmb, hmb, P<uint8_t>(sy), P<uint8_t>(su), P<uint8_t>(sv), P<uint8_t>(ry),
                             P<uint8_t>(ru), P<uint8_t>(rv), P<int>(qp), cqo, P<void>(hdr), P<int16_t>(coef),
                             P<uint8_t>(nz), P<uint8_t>(intra_flag), P<int>(intra_count), P<int>(err), use_i4x4,
                             P<int8_t>(aq), S(stream), use_i8x8, P<void>(route), nbuf, slice_rows, trellis,
                             trellis_lambda, P<int>(gprog), gprog_ints);
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("sy"), py::arg("su"), py::arg("sv"), py::arg("ry"),
     py::arg("ru"), py::arg("rv"), py::arg("qp"), py::arg("cqo"), py::arg("hdr"), py::arg("coef"), py::arg("nz"),
     py::arg("intra_flag"), py::arg("intra_count"), py::arg("err"), py::arg("use_i4x4"), py::arg("stream"),
     py::arg("aq") = 0, py::arg("use_i8x8") = 0, py::arg("route") = 0, py::arg("nbuf") = 0, py::arg("slice_rows") = 0,
     py::arg("trellis") = 0, py::arg("trellis_lambda") = 1.0f, py::arg("gprog") = 0, py::arg("gprog_ints") = 0);
  m.def("deblock", [](int B, int wmb, int hmb, uintptr_t ry, uintptr_t ru, uintptr_t rv, uintptr_t hdr, uintptr_t nz,
                      int cqo, int alpha_off, int beta_off, uintptr_t err, uintptr_t stream, uintptr_t route, int nbuf) {
    mivc_launch_deblock(B, wmb, hmb, P<uint8_t>(ry), P<uint8_t>(ru), P<uint8_t>(rv), P<void>(hdr), P<uint8_t>(nz),
                        cqo, alpha_off, beta_off, P<int>(err), S(stream), P<void>(route), nbuf);
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("ry"), py::arg("ru"), py::arg("rv"), py::arg("hdr"),
     py::arg("nz"), py::arg("cqo"), py::arg("alpha_off"), py::arg("beta_off"), py::arg("err"), py::arg("stream"),
     py::arg("route") = 0, py::arg("nbuf") = 0);
  m.def("decode_picture_dpb", [](int B, int wmb, int hmb, int dpb_n, uintptr_t y, uintptr_t u, uintptr_t v,
                                 uintptr_t cur_idx, uintptr_t reftab, uintptr_t wp, uintptr_t sub,
                                 uintptr_t hdr, uintptr_t mask, uintptr_t off, uintptr_t coef, uintptr_t run,
                                 int any_inter, int cqo, uintptr_t nz, uintptr_t err, uintptr_t stream) {
    if (dpb_n < 1 || dpb_n > 32767) throw std::invalid_argument("decode_picture_dpb: dpb_n must be 1..32767");
    mivc_launch_decode_picture_dpb(B, wmb, hmb, dpb_n, P<uint8_t>(y), P<uint8_t>(u), P<uint8_t>(v), P<int16_t>(cur_idx),
                                   P<int16_t>(reftab), P<int16_t>(wp), P<int16_t>(sub), P<void>(hdr),
                                   P<uint32_t>(mask), P<uint32_t>(off), P<int16_t>(coef), P<int8_t>(run), any_inter,
                                   cqo, P<uint8_t>(nz), P<int>(err), S(stream));
  });
  m.def("deblock_dpb", [](int B, int wmb, int hmb, int dpb_n, uintptr_t y, uintptr_t u, uintptr_t v, uintptr_t cur_idx,
                          uintptr_t hdr, uintptr_t nz, uintptr_t bs, int cqo, int alpha_off, int beta_off, uintptr_t err,
                          uintptr_t stream) {
    if (dpb_n < 1 || dpb_n > 32767) throw std::invalid_argument("deblock_dpb: dpb_n must be 1..32767");
    mivc_launch_deblock_dpb(B, wmb, hmb, dpb_n, P<uint8_t>(y), P<uint8_t>(u), P<uint8_t>(v), P<int16_t>(cur_idx),
                            P<void>(hdr), P<uint8_t>(nz), P<uint8_t>(bs), cqo, alpha_off, beta_off, P<int>(err),
                            S(stream));
  });
  m.def("scale", [](uintptr_t in, int w, int h, long long in_stride, long long in_pitch, uintptr_t out, int ow, int oh,
                    int W, int H, long long out_stride, long long out_pitch, int n, uintptr_t fx, uintptr_t cx, int tx,
                    uintptr_t fy, uintptr_t cy, int ty, int tile_w, int tile_h, int in_cols, int in_rows, int bd,
                    uintptr_t stream) {
    if (w < 1 || h < 1 || ow < 1 || oh < 1 || W < ow || H < oh || tx < 1 || ty < 1 || tile_w < 1 || tile_h < 1)
      throw std::invalid_argument("scale: bad geometry");
    return mivc_launch_scale(P<void>(in), w, h, in_stride, in_pitch, P<void>(out), ow, oh, W, H, out_stride, out_pitch,
                             n, P<int>(fx), P<int16_t>(cx), tx, P<int>(fy), P<int16_t>(cy), ty, tile_w, tile_h, in_cols,
                             in_rows, bd, S(stream));
  });
  // ---- HEVC
  m.def("hevc_prep_frame", [](int B, uintptr_t sy, uintptr_t su, uintptr_t sv, long long ss_y, long long ss_c,
                              int pitch_y, int pitch_c, int bps, int w, int h, uintptr_t dy, uintptr_t du, uintptr_t dv,
                              uintptr_t d8, int W, int H, int shift, int bd, uintptr_t stream) {
    if (mivc_launch_hevc_prep_frame(B, P<void>(sy), P<void>(su), P<void>(sv), ss_y, ss_c, pitch_y, pitch_c, bps, w, h,
                                    P<uint16_t>(dy), P<uint16_t>(du), P<uint16_t>(dv), P<uint8_t>(d8), W, H, shift, bd,
                                    S(stream)) != 0)
      throw std::invalid_argument("hevc_prep_frame: bad geometry");
  });
  m.def("hevc_proxy8", [](uintptr_t src, uintptr_t dst, long long n, int shift, uintptr_t stream) {
    if (mivc_launch_hevc_proxy8(P<uint16_t>(src), P<uint8_t>(dst), n, shift, S(stream)) != 0)
      throw std::invalid_argument("hevc_proxy8: n must be a multiple of 8");
  });
  m.def("hevc_intra", [](int B, int W, int H, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t ry, uintptr_t ru,
                         uintptr_t rv, uintptr_t ctu, uintptr_t cu, uintptr_t cy, uintptr_t cu_, uintptr_t cv,
                         uintptr_t qp, uintptr_t run, uintptr_t cand, int bd, int analyze, int recon, uintptr_t err,
                         uintptr_t stream, int sdh, uintptr_t ctb_mask, int ctu64) {
    mivc_launch_hevc_intra(B, W, H, P<uint16_t>(sy), P<uint16_t>(su), P<uint16_t>(sv), P<uint16_t>(ry), P<uint16_t>(ru),
                           P<uint16_t>(rv), P<void>(ctu), P<void>(cu), P<int16_t>(cy), P<int16_t>(cu_), P<int16_t>(cv),
                           P<int>(qp), P<int8_t>(run), P<int>(cand), bd, analyze, recon, P<int>(err), sdh,
                           P<uint8_t>(ctb_mask), S(stream), ctu64);
  }, py::arg("B"), py::arg("W"), py::arg("H"), py::arg("sy"), py::arg("su"), py::arg("sv"), py::arg("ry"), py::arg("ru"),
     py::arg("rv"), py::arg("ctu"), py::arg("cu"), py::arg("cy"), py::arg("cu_"), py::arg("cv"), py::arg("qp"),
     py::arg("run"), py::arg("cand"), py::arg("bd"), py::arg("analyze"), py::arg("recon"), py::arg("err"),
     py::arg("stream"), py::arg("sdh") = 0, py::arg("ctb_mask") = 0, py::arg("ctu64") = 0);
  m.def("hevc_inter", [](int B, int W, int H, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t fy, uintptr_t fu,
                         uintptr_t fv, uintptr_t ry, uintptr_t ru, uintptr_t rv, uintptr_t ctu, uintptr_t cu, uintptr_t cy,
                         uintptr_t cu_, uintptr_t cv, uintptr_t qp, uintptr_t run, uintptr_t cand, uintptr_t mv,
                         uintptr_t me_cost, int bd, uintptr_t stream, int tu_split, int sdh, int intra_bias,
                         uintptr_t mvb, uintptr_t dirb, uintptr_t f1y, uintptr_t f1u, uintptr_t f1v, uintptr_t wp,
                         std::vector<uintptr_t> xref, uintptr_t mv8) {
    if (dirb && (!mvb || !f1y || !f1u || !f1v)) throw std::invalid_argument("hevc_inter: B motion needs mvb and list-1 planes");
    // xref: (y, u, v) of RefPicList0[1 ..] (x265 --ref), at most 3 pictures
    if (xref.size() % 3 || xref.size() > 9) throw std::invalid_argument("hevc_inter: xref = (y, u, v) x up to 3 pictures");
    const uint16_t* xr[9] = {};
    for (size_t i = 0; i < xref.size(); ++i) xr[i] = P<uint16_t>(xref[i]);
    mivc_launch_hevc_inter(B, W, H, P<uint16_t>(sy), P<uint16_t>(su), P<uint16_t>(sv), P<uint16_t>(fy), P<uint16_t>(fu),
                           P<uint16_t>(fv), P<uint16_t>(ry), P<uint16_t>(ru), P<uint16_t>(rv), P<void>(ctu), P<void>(cu),
                           P<int16_t>(cy), P<int16_t>(cu_), P<int16_t>(cv), P<int>(qp), P<int8_t>(run), P<int>(cand),
                           P<int16_t>(mv), P<int>(me_cost), bd, tu_split, sdh, intra_bias, S(stream), P<int16_t>(mvb),
                           P<uint8_t>(dirb), P<uint16_t>(f1y), P<uint16_t>(f1u), P<uint16_t>(f1v), P<int16_t>(wp), xr,
                           P<int16_t>(mv8));
  }, py::arg("B"), py::arg("W"), py::arg("H"), py::arg("sy"), py::arg("su"), py::arg("sv"), py::arg("fy"), py::arg("fu"),
     py::arg("fv"), py::arg("ry"), py::arg("ru"), py::arg("rv"), py::arg("ctu"), py::arg("cu"), py::arg("cy"),
     py::arg("cu_"), py::arg("cv"), py::arg("qp"), py::arg("run"), py::arg("cand"), py::arg("mv"), py::arg("me_cost"),
     py::arg("bd"), py::arg("stream"), py::arg("tu_split") = 0, py::arg("sdh") = 0, py::arg("intra_bias") = 0,
     py::arg("mvb") = 0, py::arg("dirb") = 0, py::arg("f1y") = 0, py::arg("f1u") = 0, py::arg("f1v") = 0,
     py::arg("wp") = 0, py::arg("xref") = std::vector<uintptr_t>{}, py::arg("mv8") = 0);
  m.def("hevc_b", [](int mode, int B, int wmb, int hmb, uintptr_t src, uintptr_t ref0, uintptr_t ref1, uintptr_t hp0,
                     uintptr_t hp1, uintptr_t mv0, uintptr_t mv1, uintptr_t cost0, uintptr_t cost1, uintptr_t pm0,
                     uintptr_t pm1, uintptr_t tmv, uintptr_t tdir, uintptr_t mvb_in, uintptr_t dir_in, uintptr_t mvb_out,
                     uintptr_t dir_out, uintptr_t cost, uintptr_t bits, uintptr_t qp, uintptr_t aq, uintptr_t stream,
                     int bslice, int max_merge, int ctu64, uintptr_t chg_in, uintptr_t chg_out, int nref0,
                     std::vector<uintptr_t> xref, std::vector<uintptr_t> xhp, uintptr_t xmv, uintptr_t xcost,
                     uintptr_t xpm) {
    // nref0 > 1 (P pictures, x265 --ref): xref / xhp = RefPicList0[1 ..] proxies and planes; the
    // P init pass also needs the farther searches xmv / xcost / xpm
    if (nref0 < 1 || nref0 > 4) throw std::invalid_argument("hevc_b: nref0 in 1..4");
    if (nref0 > 1 && (bslice || xref.size() + 1 < static_cast<size_t>(nref0) || xhp.size() + 1 < static_cast<size_t>(nref0)))
      throw std::invalid_argument("hevc_b: nref0 > 1 needs P pictures and nref0 - 1 extra proxies / planes");
    if (nref0 > 1 && mode == 2 && (!xmv || !xcost || !xpm)) throw std::invalid_argument("hevc_b: P init with several refs needs xmv / xcost / xpm");
    const uint8_t* xr[3] = {nullptr, nullptr, nullptr};
    const uint8_t* xh[3] = {nullptr, nullptr, nullptr};
    for (int r = 0; r + 1 < nref0; ++r) {
      xr[r] = P<uint8_t>(xref[r]);
      xh[r] = P<uint8_t>(xhp[r]);
    }
    // mode 0: L0 / L1 / bi choice from the two searches; 1: one merge-aware Jacobi pass;
    // 2: a P picture's list-0 search in the same motion form
    if (mode < 0 || mode > 2) throw std::invalid_argument("hevc_b: mode 0 (choose), 1 (merge pass) or 2 (P init)");
    if (max_merge < 1 || max_merge > 5) throw std::invalid_argument("hevc_b: max_merge in 1..5");
    if (mode == 2) {
      if (!mv0 || !cost0 || !pm0 || !mvb_out || !dir_out || !cost || !bits) throw std::invalid_argument("hevc_b: P init buffers");
    } else if (!src || !ref0 || !hp0 || (bslice && (!ref1 || !hp1)) || !mvb_out || !dir_out || !cost || !bits || !qp) {
      throw std::invalid_argument("hevc_b: missing buffer");
    }
    if (mode == 0 && !bslice) throw std::invalid_argument("hevc_b: choose is for B pictures");
    if (mode == 0 && (!mv0 || !mv1 || !cost0 || !cost1 || !pm0 || !pm1)) throw std::invalid_argument("hevc_b: choose needs both searches");
    if (mode == 1 && (!mvb_in || !dir_in || mvb_in == mvb_out || dir_in == dir_out))
      throw std::invalid_argument("hevc_b: a merge pass reads and writes different motion buffers");
    if (tdir && !tmv) throw std::invalid_argument("hevc_b: tdir needs tmv");
    mivc_launch_hevc_b(mode, B, wmb, hmb, P<uint8_t>(src), P<uint8_t>(ref0), P<uint8_t>(ref1), P<uint8_t>(hp0),
                       P<uint8_t>(hp1), P<int16_t>(mv0), P<int16_t>(mv1), P<int>(cost0), P<int>(cost1), P<int16_t>(pm0),
                       P<int16_t>(pm1), P<int16_t>(tmv), P<uint8_t>(tdir), P<int16_t>(mvb_in), P<uint8_t>(dir_in),
                       P<int16_t>(mvb_out), P<uint8_t>(dir_out), P<int>(cost), P<int>(bits), P<int>(qp), P<int8_t>(aq),
                       S(stream), bslice, max_merge, ctu64, P<uint8_t>(chg_in), P<uint8_t>(chg_out), nref0,
                       xr, xh, P<int16_t>(xmv), P<int>(xcost), P<int16_t>(xpm));
  }, py::arg("mode"), py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("src"), py::arg("ref0"), py::arg("ref1"),
     py::arg("hp0"), py::arg("hp1"), py::arg("mv0"), py::arg("mv1"), py::arg("cost0"), py::arg("cost1"), py::arg("pm0"),
     py::arg("pm1"), py::arg("tmv"), py::arg("tdir"), py::arg("mvb_in"), py::arg("dir_in"), py::arg("mvb_out"),
     py::arg("dir_out"), py::arg("cost"), py::arg("bits"), py::arg("qp"), py::arg("aq"), py::arg("stream"),
     py::arg("bslice") = 1, py::arg("max_merge") = 5, py::arg("ctu64") = 0, py::arg("chg_in") = 0, py::arg("chg_out") = 0,
     py::arg("nref0") = 1, py::arg("xref") = std::vector<uintptr_t>{}, py::arg("xhp") = std::vector<uintptr_t>{},
     py::arg("xmv") = 0, py::arg("xcost") = 0, py::arg("xpm") = 0);
  m.def("hevc_deblock", [](int B, int W, int H, int bd, uintptr_t y, uintptr_t u, uintptr_t v, uintptr_t cu,
                           uintptr_t ctu, uintptr_t run, uintptr_t stream) {
    mivc_launch_hevc_deblock(B, W, H, bd, P<uint16_t>(y), P<uint16_t>(u), P<uint16_t>(v), P<void>(cu), P<void>(ctu),
                             P<int8_t>(run), S(stream));
  });
  m.def("hevc_aq", [](int B, int W, int H, int bd, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t qp,
                      float strength, uintptr_t extra, long long extra_stride, int extra_rows, uintptr_t ctb_qp,
                      uintptr_t mb_aq, uintptr_t stream) {
    if ((W & 31) || (H & 31)) throw std::invalid_argument("hevc_aq: coded size must be a multiple of 32");
    if (extra && (extra_rows < 0 || extra_rows > H / 16)) throw std::invalid_argument("hevc_aq: extra_rows out of range");
    mivc_launch_hevc_aq(B, W, H, bd, P<uint16_t>(sy), P<uint16_t>(su), P<uint16_t>(sv), P<int>(qp), strength,
                        P<float>(extra), extra_stride, extra_rows, P<int>(ctb_qp), P<int8_t>(mb_aq), S(stream));
  });
  m.def("hevc_pack_levels", [](int B, int W, int H, uintptr_t cy, uintptr_t cb, uintptr_t cr, uintptr_t nzmap,
                               uintptr_t cnt, uintptr_t off, long long cap_blocks, uintptr_t out, uintptr_t err,
                               uintptr_t stream) {
    if ((W & 31) || (H & 31)) throw std::invalid_argument("hevc_pack_levels: coded size must be a multiple of 32");
    if (cap_blocks < static_cast<long long>(W / 32) * (H / 32) * 96)
      throw std::invalid_argument("hevc_pack_levels: capacity below 96 blocks per CTB");
    mivc_launch_hevc_pack_levels(B, W, H, P<int16_t>(cy), P<int16_t>(cb), P<int16_t>(cr),
                                 P<unsigned long long>(nzmap), P<int>(cnt), P<unsigned>(off), cap_blocks,
                                 P<int16_t>(out), P<int>(err), S(stream));
  });
  m.def("hevc_merge_refine", [](int B, int wmb, int hmb, uintptr_t src, uintptr_t ref, uintptr_t hp, uintptr_t mv_in,
                                uintptr_t mv_out, uintptr_t cost, uintptr_t pm, uintptr_t qp, uintptr_t aq,
                                uintptr_t stream) {
    if (mv_in == mv_out) throw std::invalid_argument("hevc_merge_refine: mv_in and mv_out must differ (Jacobi pass)");
    if (!hp) throw std::invalid_argument("hevc_merge_refine: needs the half-sample planes");
    mivc_launch_hevc_merge_refine(B, wmb, hmb, P<uint8_t>(src), P<uint8_t>(ref), P<uint8_t>(hp), P<int16_t>(mv_in),
                                  P<int16_t>(mv_out), P<int>(cost), P<int16_t>(pm), P<int>(qp), P<int8_t>(aq), S(stream));
  });
  m.def("hevc_entropy_state_bytes", [](int W, int H) { return mivc_hevc_entropy_state_bytes(W, H); });
  // GPU CABAC slice data of B pictures of one coding step (kernels/hevc_entropy.hip); `pic` is
  // the step's hevc::CoderPic (host module hevc_coder_pic), substreams packed into pinned `dst`
  m.def("hevc_entropy", [](py::bytes pic, int B, uintptr_t qp, uintptr_t ctu, uintptr_t cu, uintptr_t col,
                           uintptr_t nzmap, uintptr_t cy, uintptr_t cb, uintptr_t cr, uintptr_t state,
                           long long state_bytes, uintptr_t out, unsigned cap, uintptr_t sizes, uintptr_t errs,
                           uintptr_t offs, uintptr_t offs_host, uintptr_t dst, unsigned long long dst_cap,
                           uintptr_t overflow, uintptr_t stream, uintptr_t prof, uintptr_t gprog, uintptr_t gctx) {
    const std::string ps = pic;
    if (ps.size() != sizeof(mivc::hevc::CoderPic)) throw std::invalid_argument("hevc_entropy: pic is not a CoderPic");
    if (!ctu || !cu || !nzmap || !cy || !cb || !cr || !state || !out || !sizes || !errs || !offs || !offs_host || !dst)
      throw std::invalid_argument("hevc_entropy: null buffer");
    if (mivc_launch_hevc_entropy(ps.data(), B, P<int>(qp), P<void>(ctu), P<void>(cu), P<void>(col),
                                 P<unsigned long long>(nzmap), P<int16_t>(cy), P<int16_t>(cb), P<int16_t>(cr),
                                 P<uint8_t>(state), state_bytes, P<uint8_t>(out), cap, P<unsigned>(sizes), P<int>(errs),
                                 P<unsigned long long>(offs), P<unsigned long long>(offs_host), P<uint8_t>(dst), dst_cap,
                                 P<int>(overflow), S(stream), P<unsigned long long>(prof), P<int>(gprog),
                                 P<void>(gctx)) != 0)
      throw std::invalid_argument("hevc_entropy: unsupported geometry (substreams <= 100, cap % 16, state size)");
  }, py::arg("pic"), py::arg("B"), py::arg("qp"), py::arg("ctu"), py::arg("cu"), py::arg("col"), py::arg("nzmap"),
     py::arg("cy"), py::arg("cb"), py::arg("cr"), py::arg("state"), py::arg("state_bytes"), py::arg("out"), py::arg("cap"),
     py::arg("sizes"), py::arg("errs"), py::arg("offs"), py::arg("offs_host"), py::arg("dst"), py::arg("dst_cap"),
     py::arg("overflow"), py::arg("stream"), py::arg("prof") = 0, py::arg("gprog") = 0, py::arg("gctx") = 0);
  m.def("hevc_qp_fixup", [](int B, int W, int H, uintptr_t ctu, uintptr_t cu, uintptr_t qp, uintptr_t run, int wpp,
                            uintptr_t stream, int ctu64) {
    mivc_launch_hevc_qp_fixup(B, W, H, P<void>(ctu), P<void>(cu), P<int>(qp), P<int8_t>(run), wpp, S(stream), ctu64);
  }, py::arg("B"), py::arg("W"), py::arg("H"), py::arg("ctu"), py::arg("cu"), py::arg("qp"), py::arg("run"),
     py::arg("wpp"), py::arg("stream"), py::arg("ctu64") = 0);
  m.def("hevc_sao", [](int B, int W, int H, int bd, uintptr_t dy, uintptr_t du, uintptr_t dv, uintptr_t y, uintptr_t u,
                       uintptr_t v, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t ctu, uintptr_t qp, uintptr_t run,
                       int enable, uintptr_t stream, int ctu64) {
    mivc_launch_hevc_sao(B, W, H, bd, P<uint16_t>(dy), P<uint16_t>(du), P<uint16_t>(dv), P<uint16_t>(y), P<uint16_t>(u),
                         P<uint16_t>(v), P<uint16_t>(sy), P<uint16_t>(su), P<uint16_t>(sv), P<void>(ctu), P<int>(qp),
                         P<int8_t>(run), enable, S(stream), ctu64);
  }, py::arg("B"), py::arg("W"), py::arg("H"), py::arg("bd"), py::arg("dy"), py::arg("du"), py::arg("dv"), py::arg("y"),
     py::arg("u"), py::arg("v"), py::arg("sy"), py::arg("su"), py::arg("sv"), py::arg("ctu"), py::arg("qp"),
     py::arg("run"), py::arg("enable"), py::arg("stream"), py::arg("ctu64") = 0);
  // HEVC decode reconstruction (hevc_decode.hip): `p` maps HevcDecParams field names to
  // ints (device pointers as data_ptr(), scalars); stage 0..5 (see the launcher)
  m.def("hevc_decode_stage", [](const py::dict& p, int stage, uintptr_t stream) {
    mivc::gpu::HevcDecParams a{};
    auto I = [&](const char* k) -> long long {
      if (!p.contains(k)) throw std::runtime_error(std::string("hevc_decode_stage: missing ") + k);
      return p[k].cast<long long>();
    };
    auto Q = [&](const char* k) -> uintptr_t { return p.contains(k) ? p[k].cast<uintptr_t>() : 0; };
    a.B = static_cast<int>(I("B"));
    a.W = static_cast<int>(I("W"));
    a.H = static_cast<int>(I("H"));
    a.D = static_cast<int>(I("D"));
    a.bd = static_cast<int>(I("bd"));
    a.bdc = static_cast<int>(I("bdc"));
    a.log2_ctb = static_cast<int>(I("log2_ctb"));
    a.wctb = static_cast<int>(I("wctb"));
    a.hctb = static_cast<int>(I("hctb"));
    const std::vector<uintptr_t> dpb = p["dpb"].cast<std::vector<uintptr_t>>();
    const std::vector<uintptr_t> res = p["res"].cast<std::vector<uintptr_t>>();
    const std::vector<uintptr_t> tmp = p["tmp"].cast<std::vector<uintptr_t>>();
    for (int c = 0; c < 3; ++c) {
      a.dpb[c] = reinterpret_cast<uint16_t*>(dpb.at(c));
      a.res[c] = reinterpret_cast<int16_t*>(res.at(c));
      a.tmp[c] = reinterpret_cast<uint16_t*>(tmp.at(c));
    }
    a.cur = P<int8_t>(Q("cur"));
    a.reftab = P<int8_t>(Q("reftab"));
    a.run = P<int8_t>(Q("run"));
    a.meta = P<int32_t>(Q("meta"));
    a.mvf = P<uint8_t>(Q("mvf"));
    a.mvf_sub = P<uint8_t>(Q("mvf_sub"));
    a.bs = P<uint8_t>(Q("bs"));
    a.ctbs = P<uint8_t>(Q("ctbs"));
    a.sao = P<uint8_t>(Q("sao"));
    a.tus = P<uint8_t>(Q("tus"));
    a.tu_base = P<int32_t>(Q("tu_base"));
    a.coefs = P<int16_t>(Q("coefs"));
    a.coef_base = P<int64_t>(Q("coef_base"));
    a.ops = P<uint8_t>(Q("ops"));
    a.op_base = P<int32_t>(Q("op_base"));
    a.ctb_ops = P<uint32_t>(Q("ctb_ops"));
    a.refs = P<uint8_t>(Q("refs"));
    a.ref_base = P<int32_t>(Q("ref_base"));
    a.slices = P<uint8_t>(Q("slices"));
    a.slice_base = P<int32_t>(Q("slice_base"));
    a.scaling = P<uint8_t>(Q("scaling"));
    a.max_tus = static_cast<int>(I("max_tus"));
    a.err = P<int>(Q("err"));
    if (p.contains("out")) {
      const std::vector<uintptr_t> out = p["out"].cast<std::vector<uintptr_t>>();
      for (int c = 0; c < 3; ++c) a.out[c] = reinterpret_cast<void*>(out.at(c));
      a.out_u8 = static_cast<int>(I("out_u8"));
      a.Fo = static_cast<int>(I("Fo"));
      a.out_w = static_cast<int>(I("out_w"));
      a.out_h = static_cast<int>(I("out_h"));
      a.crop_x = static_cast<int>(I("crop_x"));
      a.crop_y = static_cast<int>(I("crop_y"));
      a.disp = P<int16_t>(Q("disp"));
    }
    if (!a.cur || !a.run || !a.meta || !a.mvf || !a.err) throw std::runtime_error("hevc_decode_stage: null pointer");
    const int r = mivc_launch_hevc_decode(&a, stage, S(stream));
    if (r != 0) throw std::runtime_error("hevc_decode_stage: launch failed (" + std::to_string(r) + ")");
  });
  m.def("cavlc_mb_bytes", []() { return mivc_cavlc_mb_bytes(); });
  m.def("cabac_nb_bytes", []() { return mivc_cabac_nb_bytes(); });
  m.def("cabac_gap", []() { return mivc_cabac_gap(); });
  m.def("cabac_bin", [](int B, int wmb, int hmb, uintptr_t hdr, uintptr_t coef, uintptr_t mask, uintptr_t nb,
                        uintptr_t cnt, uintptr_t off, uintptr_t tot, uintptr_t pool, long long pool_cap,
                        uintptr_t pool_used, uintptr_t base, uintptr_t total, uintptr_t slot_qp, int slice_type,
                        int num_ref_l0, int num_ref_l1, int t8x8_mode, uintptr_t err, uintptr_t stream, uintptr_t route,
                        int slice_rows) {
    if ((pool & 15) != 0) throw std::invalid_argument("cabac_bin: symbol pool must be 16-byte aligned");
    if (B < 1 || wmb < 1 || hmb < 1) throw std::invalid_argument("cabac_bin: bad geometry");
    mivc_launch_cabac_bin(B, wmb, hmb, P<void>(hdr), P<int16_t>(coef), P<uint32_t>(mask), P<void>(nb), P<int>(cnt),
                          P<long long>(off), P<int>(tot), P<uint16_t>(pool), pool_cap, P<long long>(pool_used),
                          P<long long>(base), P<int>(total), P<int>(slot_qp), slice_type, num_ref_l0, num_ref_l1,
                          t8x8_mode, P<int>(err), S(stream), P<void>(route), slice_rows);
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("hdr"), py::arg("coef"), py::arg("mask"), py::arg("nb"),
     py::arg("cnt"), py::arg("off"), py::arg("tot"), py::arg("pool"), py::arg("pool_cap"), py::arg("pool_used"),
     py::arg("base"), py::arg("total"), py::arg("slot_qp"), py::arg("slice_type"), py::arg("num_ref_l0"),
     py::arg("num_ref_l1"), py::arg("t8x8_mode"), py::arg("err"), py::arg("stream"), py::arg("route") = 0,
     py::arg("slice_rows") = 0);
  m.def("cabac_code", [](int L, int B, uintptr_t pool, uintptr_t base, uintptr_t total, uintptr_t hdr_bits,
                         uintptr_t hdr_nbits, uintptr_t slot_qp, unsigned long long itypes, uintptr_t bytes,
                         uintptr_t out, uintptr_t out_off, uintptr_t err, uintptr_t stream, uintptr_t host_out,
                         long long host_cap) {
    if (B < 1 || L < 1 || L % B != 0 || L / B > 64) throw std::invalid_argument("cabac_code: L must be G * B, G <= 64");
    if ((out & 15) || (host_out & 15)) throw std::invalid_argument("cabac_code: output buffers must be 16-byte aligned");
    mivc_launch_cabac_code(L, B, P<uint16_t>(pool), P<long long>(base), P<int>(total), P<uint32_t>(hdr_bits),
                           P<int>(hdr_nbits), P<int>(slot_qp), itypes, P<int>(bytes), P<uint8_t>(out),
                           P<long long>(out_off), P<int>(err), P<uint8_t>(host_out), host_cap, S(stream));
  });
  m.def("cavlc", [](int B, int wmb, int hmb, uintptr_t hdr, uintptr_t coef, uintptr_t mbs, uintptr_t len, uintptr_t off,
                    uintptr_t trail, uintptr_t total_bits, uintptr_t slot_bytes, uintptr_t words, long long cap_words,
                    uintptr_t hdr_bits, uintptr_t hdr_nbits, int pslice, int slice_qp, uintptr_t slot_qp,
                    uintptr_t out, uintptr_t out_off, uintptr_t stream, uintptr_t nz) {
    mivc_launch_cavlc(B, wmb, hmb, P<void>(hdr), P<int16_t>(coef), P<void>(mbs), P<int>(len), P<long long>(off),
                      P<int>(trail), P<long long>(total_bits), P<int>(slot_bytes), P<uint32_t>(words), cap_words,
                      P<uint32_t>(hdr_bits), P<int>(hdr_nbits), pslice, slice_qp, P<int>(slot_qp), P<uint8_t>(out),
                      P<long long>(out_off), P<uint8_t>(nz), S(stream));
  }, py::arg("B"), py::arg("wmb"), py::arg("hmb"), py::arg("hdr"), py::arg("coef"), py::arg("mbs"), py::arg("len"),
     py::arg("off"), py::arg("trail"), py::arg("total_bits"), py::arg("slot_bytes"), py::arg("words"),
     py::arg("cap_words"), py::arg("hdr_bits"), py::arg("hdr_nbits"), py::arg("pslice"), py::arg("slice_qp"),
     py::arg("slot_qp"), py::arg("out"), py::arg("out_off"), py::arg("stream"), py::arg("nz") = 0);
  m.def("sse", [](int B, int W, int H, int w, int h, uintptr_t sy, uintptr_t su, uintptr_t sv, uintptr_t ry,
                  uintptr_t ru, uintptr_t rv, uintptr_t sse, uintptr_t ssim, uintptr_t stream, uintptr_t route, int nbuf) {
    mivc_launch_sse(B, W, H, w, h, P<uint8_t>(sy), P<uint8_t>(su), P<uint8_t>(sv), P<uint8_t>(ry), P<uint8_t>(ru),
                    P<uint8_t>(rv), P<unsigned long long>(sse), P<float>(ssim), S(stream), P<void>(route), nbuf);
  }, py::arg("B"), py::arg("W"), py::arg("H"), py::arg("w"), py::arg("h"), py::arg("sy"), py::arg("su"), py::arg("sv"),
     py::arg("ry"), py::arg("ru"), py::arg("rv"), py::arg("sse"), py::arg("ssim"), py::arg("stream"),
     py::arg("route") = 0, py::arg("nbuf") = 0);
  m.def("satd_blocks", [](uintptr_t src, uintptr_t pred, uintptr_t out, int n, int mode, uintptr_t stream) {
    if (n <= 0) throw std::invalid_argument("satd_blocks: n must be positive");
    mivc_launch_satd_blocks(P<uint8_t>(src), P<uint8_t>(pred), P<int>(out), n, mode, S(stream));
  });
  m.def("trellis_blocks", [](uintptr_t w, uintptr_t out, int n, int qp, int mode, int skip_dc, uintptr_t stream) {
    if (n <= 0 || qp < 0 || qp > 51) throw std::invalid_argument("trellis_blocks: n > 0, 0 <= qp <= 51");
    mivc_launch_trellis_blocks(P<int>(w), P<int>(out), n, qp, mode, skip_dc, S(stream));
  });
  m.def("lookahead_low_bytes", [](int w, int h, int n) { return mivc_lookahead_low_bytes(w, h, n); });
  m.def("lookahead_quarter_bytes", [](int w, int h, int n) { return mivc_lookahead_quarter_bytes(w, h, n); });
  m.def("lookahead_multi", [](uintptr_t low, int w, int h, int n, int f, uintptr_t blk_cost, uintptr_t blk_mv, int D,
                              int range, uintptr_t out, uintptr_t stream, uintptr_t wt) {
    const int r = mivc_launch_lookahead_multi(P<uint8_t>(low), w, h, n, f, P<int>(blk_cost), P<int>(blk_mv), D, range,
                                              P<unsigned long long>(out), S(stream), P<float>(wt));
    if (r != 0) throw std::invalid_argument("lookahead_multi: bad arguments (" + std::to_string(r) + ")");
  }, py::arg("low"), py::arg("w"), py::arg("h"), py::arg("n"), py::arg("f"), py::arg("blk_cost"), py::arg("blk_mv"),
     py::arg("D"), py::arg("range"), py::arg("out"), py::arg("stream"), py::arg("wt") = 0);
  m.def("lookahead", [](uintptr_t y, int w, int h, long long fstride, int n, int f, uintptr_t low, uintptr_t frame_cost,
                        uintptr_t blk_cost, int range, uintptr_t stream, uintptr_t blk_mv, uintptr_t low4, uintptr_t mv4,
                        uintptr_t cost4, uintptr_t wt, uintptr_t wstats, float thr_mean, float thr_scale, int stage) {
    int rc = mivc_launch_lookahead(P<uint8_t>(y), w, h, fstride, n, f, P<uint8_t>(low),
                                   P<unsigned long long>(frame_cost), P<int>(blk_cost), P<int>(blk_mv), range,
                                   S(stream), P<uint8_t>(low4), P<int>(mv4), P<unsigned long long>(cost4), P<float>(wt),
                                   P<unsigned long long>(wstats), thr_mean, thr_scale, stage);
    if (rc != 0) throw std::invalid_argument("lookahead: bad geometry or range (4, 6, 8)");
  }, py::arg("y"), py::arg("w"), py::arg("h"), py::arg("fstride"), py::arg("n"), py::arg("f"), py::arg("low"),
     py::arg("frame_cost"), py::arg("blk_cost"), py::arg("range"), py::arg("stream"), py::arg("blk_mv") = 0,
     py::arg("low4") = 0, py::arg("mv4") = 0, py::arg("cost4") = 0, py::arg("wt") = 0, py::arg("wstats") = 0,
     py::arg("thr_mean") = 2.0f, py::arg("thr_scale") = 0.08f, py::arg("stage") = 3);
}
