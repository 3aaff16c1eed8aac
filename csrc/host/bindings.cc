// pybind11 bindings of the host (CPU) native library: bitstream primitives,
// CAVLC writer, independent decoder, CPU reference encoder, Annex-B tools.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "../common/h264_enc_math.h"
#include "annexb.h"
#include "cabac_writer.h"
#include "cavlc_writer.h"
#include "cpu_encoder.h"
#include "decode_batch.h"
#include "h264_decoder.h"
#include "hevc_codec.h"
#include "hevc_dec.h"
#include "lowres.h"

namespace mivc {
int selftest_i4_taps(int trials, uint32_t seed);
namespace hevc {
std::vector<uint8_t> hevc_exercise(uint32_t seed);
}
}

namespace py = pybind11;
using namespace mivc;
using namespace mivc::h264;

namespace {

py::bytes to_bytes(const std::vector<uint8_t>& v) {
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}

template <class T>
T dget(const py::dict& d, const char* k, T def) {
  if (d.contains(k)) return d[k].cast<T>();
  return def;
}

EncoderConfig cfg_from(const py::dict& d) {
  EncoderConfig c;
  c.width = dget<int>(d, "width", 0);
  c.height = dget<int>(d, "height", 0);
  c.fps = dget<double>(d, "fps", 30.0);
  c.qp = dget<int>(d, "qp", 26);
  c.crf = dget<double>(d, "crf", -1.0);
  c.keyint = dget<int>(d, "keyint", 250);
  c.me_range = dget<int>(d, "me_range", 16);
  c.subpel = dget<int>(d, "subpel", 2);
  c.use_i4x4 = dget<int>(d, "i4x4", 1);
  c.deblock = dget<int>(d, "deblock", 1);
  c.chroma_qp_offset = dget<int>(d, "chroma_qp_offset", 0);
  c.vui = dget<int>(d, "vui", 1);
  c.cabac = dget<int>(d, "cabac", 0);
  c.t8x8 = dget<int>(d, "t8x8", 0);
  c.bframes = dget<int>(d, "bframes", 0);
  c.pyramid = dget<int>(d, "pyramid", 0);
  c.refs = dget<int>(d, "refs", 1);
  c.weighted_bipred = dget<int>(d, "weighted_bipred", 0);
  c.weightp = dget<int>(d, "weightp", 0);
  c.constrained_intra = dget<int>(d, "constrained_intra", 0);
  c.level_idc = dget<int>(d, "level_idc", 0);
  c.bit_depth = dget<int>(d, "bit_depth", 8);
  if (c.bit_depth < 8 || c.bit_depth > 14) throw std::runtime_error("bit_depth in 8..14");
  c.bit_depth_chroma = dget<int>(d, "bit_depth_chroma", 0);
  if (c.bit_depth_chroma != 0 && (c.bit_depth_chroma < 8 || c.bit_depth_chroma > 14))
    throw std::runtime_error("bit_depth_chroma in 8..14");
  c.cqm = dget<int>(d, "cqm", 0);
  c.cqm_coded = dget<int>(d, "cqm_coded", 0xFF);
  if (c.cqm < 0 || c.cqm > 3) throw std::runtime_error("cqm in 0..3");
  if (d.contains("cqm4")) {  // [6, 16] raster weights
    auto a = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>::ensure(d["cqm4"]);
    if (!a || a.size() != 96) throw std::runtime_error("cqm4: 6 x 16 weights");
    std::memcpy(c.cqm4, a.data(), 96);
  }
  if (d.contains("cqm8")) {  // [2, 64]
    auto a = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>::ensure(d["cqm8"]);
    if (!a || a.size() != 128) throw std::runtime_error("cqm8: 2 x 64 weights");
    std::memcpy(c.cqm8, a.data(), 128);
  }
  if (c.refs < 1 || c.refs > 16) throw std::runtime_error("refs must be in 1..16");
  return c;
}

py::dict picture_to_dict(const DecodedPicture& p) {
  py::dict d;
  d["width"] = p.width;
  d["height"] = p.height;
  d["coded_width"] = p.coded_width;
  d["coded_height"] = p.coded_height;
  d["frame_num"] = p.frame_num;
  d["poc"] = p.poc;
  d["idr"] = p.idr;
  d["slice_type"] = p.slice_type;
  d["bit_depth"] = p.bit_depth;
  auto planes = [&](auto tag, const auto& i420, const auto& y, const auto& u, const auto& v) {
    using T = decltype(tag);
    py::array_t<T> a(static_cast<py::ssize_t>(i420.size()));
    std::memcpy(a.mutable_data(), i420.data(), i420.size() * sizeof(T));
    d["i420"] = a;
    py::array_t<T> ya({p.coded_height, p.coded_width});
    std::memcpy(ya.mutable_data(), y.data(), y.size() * sizeof(T));
    d["y_coded"] = ya;
    py::array_t<T> ua({p.coded_height / 2, p.coded_width / 2});
    std::memcpy(ua.mutable_data(), u.data(), u.size() * sizeof(T));
    d["u_coded"] = ua;
    py::array_t<T> va({p.coded_height / 2, p.coded_width / 2});
    std::memcpy(va.mutable_data(), v.data(), v.size() * sizeof(T));
    d["v_coded"] = va;
  };
  if (p.bit_depth > 8) planes(uint16_t{}, p.cropped_i420_16(), p.y16, p.u16, p.v16);  // High 10: uint16 planes
  else planes(uint8_t{}, p.cropped_i420(), p.y, p.u, p.v);
  py::array_t<int8_t> k(static_cast<py::ssize_t>(p.mb_kind.size()));
  std::memcpy(k.mutable_data(), p.mb_kind.data(), p.mb_kind.size());
  d["mb_kind"] = k;
  py::array_t<int8_t> q(static_cast<py::ssize_t>(p.mb_qp.size()));
  std::memcpy(q.mutable_data(), p.mb_qp.data(), p.mb_qp.size());
  d["mb_qp"] = q;
  py::array_t<int16_t> mv(static_cast<py::ssize_t>(p.mv.size()));
  if (!p.mv.empty()) std::memcpy(mv.mutable_data(), p.mv.data(), p.mv.size() * 2);
  d["mv"] = mv;
  return d;
}

using ParsedSegment = H264Parsed;  // decode_batch.h

template <class T>
py::array_t<T> vec_array(const std::vector<std::vector<T>*>& parts, std::vector<py::ssize_t> shape) {
  py::array_t<T> a(shape);
  T* d = a.mutable_data();
  for (const std::vector<T>* v : parts) {
    if (!v->empty()) std::memcpy(d, v->data(), v->size() * sizeof(T));
    d += v->size();
  }
  return a;
}

// meta [P, 12] (decode order) of the parsed pictures; columns as in segment_to_dict
py::array_t<int32_t> segment_meta(const ParsedSegment& seg) {
  const py::ssize_t P = static_cast<py::ssize_t>(seg.pics.size());
  py::array_t<int32_t> meta({P, static_cast<py::ssize_t>(12)});
  int32_t* mt = meta.mutable_data();
  for (py::ssize_t i = 0; i < P; ++i) {
    const DecodedPicture& p = seg.pics[i];
    const int32_t v[12] = {p.pic_id, p.ref_id, p.nal_ref, p.idr, p.slice_type, p.slice_qp, p.alpha_off, p.beta_off,
                           p.chroma_qp_offset, p.deblock, p.gpu_ok ? 1 : 0, p.poc};
    std::copy(v, v + 12, mt + i * 12);
  }
  return meta;
}

// the small tables of a parsed segment for the GPU decoder's planning (no per-MB records)
py::dict segment_info(const ParsedSegment& seg) {
  py::dict d;
  d["error"] = seg.error.empty() ? py::object(py::none()) : py::object(py::str(seg.error));
  const py::ssize_t P = static_cast<py::ssize_t>(seg.pics.size());
  d["n"] = seg.error.empty() ? P : 0;
  if (!seg.error.empty() || P == 0) return d;
  const DecodedPicture& p0 = seg.pics[0];
  d["width"] = p0.width;
  d["height"] = p0.height;
  d["coded_width"] = p0.coded_width;
  d["coded_height"] = p0.coded_height;
  d["crop_x"] = p0.crop_x;
  d["crop_y"] = p0.crop_y;
  bool same = true;
  for (const DecodedPicture& p : seg.pics)
    same = same && p.coded_width == p0.coded_width && p.coded_height == p0.coded_height &&
           p.bs.size() == p0.blk_mask.size() * 16 && p.list_ids.size() == 64;
  if (!same) {
    d["error"] = std::string("resolution changes inside the segment");
    d["n"] = 0;
    return d;
  }
  d["meta"] = segment_meta(seg);
  py::array_t<int32_t> lists({P, static_cast<py::ssize_t>(2), static_cast<py::ssize_t>(32)});
  for (py::ssize_t i = 0; i < P; ++i) std::memcpy(lists.mutable_data() + i * 64, seg.pics[i].list_ids.data(), 64 * 4);
  d["lists"] = lists;
  return d;
}

py::dict segment_to_dict(ParsedSegment& seg) {
  py::dict d;
  if (!seg.error.empty()) {
    d["error"] = seg.error;
    return d;
  }
  d["error"] = py::none();
  const py::ssize_t P = static_cast<py::ssize_t>(seg.pics.size());
  d["n"] = P;
  if (P == 0) return d;
  const DecodedPicture& p0 = seg.pics[0];
  const py::ssize_t nmb = static_cast<py::ssize_t>(p0.blk_mask.size());
  d["width"] = p0.width;
  d["height"] = p0.height;
  d["coded_width"] = p0.coded_width;
  d["coded_height"] = p0.coded_height;
  d["crop_x"] = p0.crop_x;
  d["crop_y"] = p0.crop_y;
  std::vector<std::vector<uint8_t>*> hdr;
  std::vector<std::vector<uint32_t>*> mask, off;
  std::vector<std::vector<int16_t>*> coef, subs, wps;
  std::vector<std::vector<uint8_t>*> bss;
  std::vector<std::vector<int32_t>*> lists;
  py::array_t<int64_t> pic_off(P + 1);
  py::array_t<int64_t> sub_off(P + 1);
  int64_t* so = sub_off.mutable_data();
  so[0] = 0;
  py::array_t<int32_t> meta({P, static_cast<py::ssize_t>(12)});
  int64_t* po = pic_off.mutable_data();
  int32_t* mt = meta.mutable_data();
  po[0] = 0;
  bool same_geom = true;
  for (py::ssize_t i = 0; i < P; ++i) {
    DecodedPicture& p = seg.pics[i];
    same_geom = same_geom && p.coded_width == p0.coded_width && p.coded_height == p0.coded_height &&
                static_cast<py::ssize_t>(p.blk_mask.size()) == nmb;
    same_geom = same_geom && p.bs.size() == static_cast<size_t>(nmb) * 16 &&
                p.wp.size() == static_cast<size_t>(kWpEntries) && p.list_ids.size() == 64;
    hdr.push_back(&p.hdr);
    subs.push_back(&p.sub);
    so[i + 1] = so[i] + static_cast<int64_t>(p.sub.size() / kSubEntry);
    bss.push_back(&p.bs);
    lists.push_back(&p.list_ids);
    wps.push_back(&p.wp);
    mask.push_back(&p.blk_mask);
    off.push_back(&p.blk_off);
    coef.push_back(&p.coef);
    po[i + 1] = po[i] + static_cast<int64_t>(p.coef.size() / 16);
    int32_t* m = mt + i * 12;
    m[0] = p.pic_id;
    m[1] = p.ref_id;
    m[2] = p.nal_ref;
    m[3] = p.idr;
    m[4] = p.slice_type;
    m[5] = p.slice_qp;
    m[6] = p.alpha_off;
    m[7] = p.beta_off;
    m[8] = p.chroma_qp_offset;
    m[9] = p.deblock;
    m[10] = p.gpu_ok ? 1 : 0;
    m[11] = p.poc;
  }
  if (!same_geom) {
    d["error"] = std::string("resolution changes inside the segment");
    return d;
  }
  d["hdr"] = vec_array<uint8_t>(hdr, {P, nmb, static_cast<py::ssize_t>(sizeof(MbHeader))});
  d["mask"] = vec_array<uint32_t>(mask, {P, nmb});
  d["off"] = vec_array<uint32_t>(off, {P, nmb});
  d["coef"] = vec_array<int16_t>(coef, {static_cast<py::ssize_t>(po[P] * 16)});
  d["pic_off"] = pic_off;
  d["meta"] = meta;
  d["sub"] = vec_array<int16_t>(subs, {static_cast<py::ssize_t>(so[P] * kSubEntry)});
  d["sub_off"] = sub_off;
  d["bs"] = vec_array<uint8_t>(bss, {P, nmb, 16});
  d["lists"] = vec_array<int32_t>(lists, {P, 2, 32});
  d["wp"] = vec_array<int16_t>(wps, {P, static_cast<py::ssize_t>(kWpEntries)});
  return d;
}

// Slice header of one picture from the frame-parameter dict: idr, slice_type, frame_num,
// idr_pic_id, qp, poc (POC type 0), nal_ref_idc, num_ref (L0 / L1 active), direct_spatial.
SliceHeader slice_header_from(const EncoderConfig& c, const SPS& sps, const PPS& pps, const py::dict& fp) {
  SliceHeader sh;
  bool idr = dget<int>(fp, "idr", 0) != 0;
  sh.nal_unit_type = idr ? NAL_IDR : NAL_SLICE;
  sh.slice_type = dget<int>(fp, "slice_type", idr ? SLICE_I : SLICE_P);
  sh.nal_ref_idc = dget<int>(fp, "nal_ref_idc", idr ? 3 : (sh.slice_type == SLICE_B ? 0 : 2));
  sh.frame_num = dget<int>(fp, "frame_num", 0);
  sh.idr_pic_id = dget<int>(fp, "idr_pic_id", 0);
  sh.poc_lsb = dget<int>(fp, "poc", 0);
  sh.slice_qp_delta = dget<int>(fp, "qp", 26) - pps.pic_init_qp;
  sh.disable_deblocking_filter_idc = c.deblock ? 0 : 1;
  sh.num_ref_idx_l0_active = dget<int>(fp, "num_ref_l0", pps.num_ref_idx_l0_default);
  sh.num_ref_idx_l1_active = dget<int>(fp, "num_ref_l1", pps.num_ref_idx_l1_default);
  sh.num_ref_idx_override = (sh.num_ref_idx_l0_active != pps.num_ref_idx_l0_default ||
                             sh.num_ref_idx_l1_active != pps.num_ref_idx_l1_default) ? 1 : 0;
  sh.direct_spatial = dget<int>(fp, "direct_spatial", 1);
  sh.first_mb = dget<int>(fp, "first_mb", 0);  // several slices per picture: each writes its MB range
  // ref_pic_list_modification of list 0 / 1: [(modification_of_pic_nums_idc, abs_diff_pic_num_minus1
  // or long_term_pic_num), ...] (the encoder's POC-distance order where the default PicNum order
  // differs: a P picture after a reference B); mmco: [(op, value), ...] adaptive marking
  for (int l = 0; l < 2; ++l) {
    const char* key = l ? "mod_l1" : "mod_l0";
    if (!fp.contains(key) || fp[key].is_none()) continue;
    for (auto& e : fp[key].cast<std::vector<std::pair<int, int>>>()) {
      if (e.first < 0 || e.first > 2 || e.second < 0) throw std::runtime_error("ref_pic_list_modification: bad entry");
      sh.mods[l].push_back(RefMod{e.first, e.second});
    }
  }
  if (fp.contains("mmco") && !fp["mmco"].is_none()) {
    for (auto& e : fp["mmco"].cast<std::vector<std::pair<int, int>>>()) {
      if (e.first != 1) throw std::runtime_error("mmco: only operation 1 (unmark a short-term picture) is written");
      Mmco m{};
      m.op = 1;
      m.diff_minus1 = e.second;
      sh.mmco.push_back(m);
    }
    sh.adaptive_ref_pic_marking = sh.mmco.empty() ? 0 : 1;
  }
  sh.cabac_init_idc = 0;
  // explicit weights of RefPicList0[0] (P slices of a weighted_pred_flag PPS): [luma log2
  // denominator, chroma log2 denominator, luma weight, offset, Cb weight, offset, Cr weight,
  // offset]; every other reference keeps the default weights
  if (fp.contains("wp") && !fp["wp"].is_none()) {
    auto v = fp["wp"].cast<std::vector<int>>();
    if (v.size() != 8) throw std::runtime_error("wp: 8 values (denominators, luma w/o, Cb w/o, Cr w/o)");
    WeightTable& w = sh.wt;
    w.luma_log2 = v[0];
    w.chroma_log2 = v[1];
    if (w.luma_log2 < 0 || w.luma_log2 > 7 || w.chroma_log2 < 0 || w.chroma_log2 > 7)
      throw std::runtime_error("wp: log2 denominators in 0..7");
    for (int i = 2; i < 8; ++i)
      if (v[i] < -128 || v[i] > 127) throw std::runtime_error("wp: weights and offsets in -128..127");
    w.lw[0][0] = v[2];
    w.lo[0][0] = v[3];
    w.cw[0][0][0] = v[4];
    w.co[0][0][0] = v[5];
    w.cw[0][0][1] = v[6];
    w.co[0][0][1] = v[7];
    w.lflag[0][0] = v[2] != (1 << v[0]) || v[3] != 0;
    w.cflag[0][0] = v[4] != (1 << v[1]) || v[5] != 0 || v[6] != (1 << v[1]) || v[7] != 0;
    sh.has_weights = true;
  }
  (void)sps;
  return sh;
}

hevc::HevcConfig hevc_cfg_from(const py::dict& d) {
  hevc::HevcConfig c;
  c.width = dget<int>(d, "width", 0);
  c.height = dget<int>(d, "height", 0);
  c.bit_depth = dget<int>(d, "bit_depth", 8);
  c.fps = dget<double>(d, "fps", 30.0);
  c.sao = dget<int>(d, "sao", 1);
  c.deblock = dget<int>(d, "deblock", 1);
  c.max_merge = dget<int>(d, "max_merge", 5);
  c.wpp = dget<int>(d, "wpp", 0);
  c.threads = dget<int>(d, "threads", 1);
  c.cu_qp_delta = dget<int>(d, "cu_qp_delta", 0);
  c.tu_inter_depth = dget<int>(d, "tu_inter_depth", 0);
  c.sdh = dget<int>(d, "sdh", 0);
  c.level_idc = dget<int>(d, "level_idc", 0);
  c.bframes = dget<int>(d, "bframes", 0);
  c.tmvp = dget<int>(d, "tmvp", 0);
  c.pyramid = dget<int>(d, "pyramid", 0);
  c.ctu64 = dget<int>(d, "ctu64", 0);
  c.weightp = dget<int>(d, "weightp", 0);
  c.refs = dget<int>(d, "refs", 1);
  if (c.refs < 1 || c.refs > hevc::kMaxRefs) throw std::runtime_error("HEVC: refs in 1..4");
  if (c.tu_inter_depth < 0 || c.tu_inter_depth > 1) throw std::runtime_error("HEVC: tu_inter_depth in 0..1");
  if (c.threads < 1 || c.threads > 256) throw std::runtime_error("HEVC: threads in 1..256");
  if (c.width <= 0 || c.height <= 0 || (c.width & 1) || (c.height & 1)) throw std::runtime_error("HEVC: bad size");
  if (c.bit_depth != 8 && c.bit_depth != 10) throw std::runtime_error("HEVC: bit_depth must be 8 or 10");
  if (c.max_merge < 1 || c.max_merge > 5) throw std::runtime_error("HEVC: max_merge in 1..5");
  return c;
}

template <class T>
py::array_t<T> to_array(const std::vector<T>& v, std::vector<py::ssize_t> shape) {
  py::array_t<T> a(shape);
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

py::dict hevc_picture_to_dict(const hevc::HevcPicture& p) {
  py::dict d;
  d["width"] = p.width;
  d["height"] = p.height;
  d["coded_width"] = p.coded_width;
  d["coded_height"] = p.coded_height;
  d["bit_depth"] = p.bit_depth;
  d["poc"] = p.poc;
  d["idr"] = p.idr;
  d["slice_type"] = p.slice_type;
  d["qp"] = p.qp;
  const py::ssize_t H = p.coded_height, W = p.coded_width;
  d["y"] = to_array(p.y, {H, W});
  d["u"] = to_array(p.u, {H / 2, W / 2});
  d["v"] = to_array(p.v, {H / 2, W / 2});
  std::vector<uint8_t> ctu(p.ctu.size() * sizeof(hevc::CtuInfo)), cu(p.cu.size() * sizeof(hevc::CuInfo));
  if (!ctu.empty()) std::memcpy(ctu.data(), p.ctu.data(), ctu.size());
  if (!cu.empty()) std::memcpy(cu.data(), p.cu.data(), cu.size());
  d["ctu"] = to_array(ctu, {static_cast<py::ssize_t>(p.ctu.size()), static_cast<py::ssize_t>(sizeof(hevc::CtuInfo))});
  d["cu"] = to_array(cu, {static_cast<py::ssize_t>(p.cu.size()), static_cast<py::ssize_t>(sizeof(hevc::CuInfo))});
  d["coef_y"] = to_array(p.coef_y, {H, W});
  d["coef_cb"] = to_array(p.coef_cb, {H / 2, W / 2});
  d["coef_cr"] = to_array(p.coef_cr, {H / 2, W / 2});
  return d;
}


// general HEVC decoder output -> dict (decoding order; "display" = output position or -1)
template <class T>
py::array_t<uint8_t> raw_rows(const std::vector<T>& v) {
  py::array_t<uint8_t> a({static_cast<py::ssize_t>(v.size()), static_cast<py::ssize_t>(sizeof(T))});
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

py::dict dec_picture_to_dict(const hevc::DecPicture& p, bool recon) {
  py::dict d;
  d["decode_idx"] = p.decode_idx;
  d["poc"] = p.poc;
  d["cvs"] = p.cvs;
  d["output"] = p.output;
  d["irap"] = p.irap;
  d["idr"] = p.idr;
  d["nal_type"] = p.nal_type;
  d["slice_type"] = p.slice_type;
  d["qp"] = p.slice_qp;
  d["coded_width"] = p.W;
  d["coded_height"] = p.H;
  d["width"] = p.width;
  d["height"] = p.height;
  d["crop_x"] = p.crop_x;
  d["crop_y"] = p.crop_y;
  d["bit_depth"] = p.bit_depth;
  d["log2_ctb"] = p.log2_ctb;
  if (recon && !p.y.empty()) {
    const py::ssize_t H = p.H, W = p.W;
    d["y"] = to_array(p.y, {H, W});
    d["u"] = to_array(p.u, {H / 2, W / 2});
    d["v"] = to_array(p.v, {H / 2, W / 2});
  }
  return d;
}

// GPU hand-off records of one segment: every array concatenated over its pictures
// (decoding order) with per-picture offsets; record layouts of csrc/host/hevc_dec.h
py::dict dec_segment_records(std::vector<hevc::DecPicture>& pics, const std::vector<int>& order) {
  py::dict d;
  const size_t P = pics.size();
  if (P == 0) {
    d["n"] = 0;
    return d;
  }
  const hevc::DecPicture& f = pics[0];
  const int w4 = f.W / 4, h4 = f.H / 4, nctb = f.wctb * f.hctb;
  std::vector<int32_t> meta(P * 24, 0), ref_ids(P * 16, -1), display(P, -1);
  for (size_t i = 0; i < order.size(); ++i) display[order[i]] = static_cast<int32_t>(i);
  std::vector<uint8_t> mvf, mvf_sub, bs, ctbs, sao, scaling;
  std::vector<int64_t> mvf_sub_off(P + 1, 0);
  std::vector<hevc::DecTu> tus;
  std::vector<hevc::DecIntraOp> ops;
  std::vector<hevc::DecRefEntry> refs;
  std::vector<hevc::DecSlice> slices;
  std::vector<int16_t> coefs;
  std::vector<int64_t> tu_off(P + 1), op_off(P + 1), ref_off(P + 1), slice_off(P + 1), coef_off(P + 1);
  std::vector<uint32_t> ctb_ops(P * (nctb + 1));
  mvf.reserve(P * (w4 / 2) * (h4 / 2) * 12);
  for (size_t i = 0; i < P; ++i) {
    hevc::DecPicture& p = pics[i];
    if (p.W != f.W || p.H != f.H || p.log2_ctb != f.log2_ctb || p.bit_depth != f.bit_depth)
      throw std::runtime_error("HEVC segment changes geometry / bit depth between pictures");
    int32_t* m = &meta[i * 24];
    const int vals[24] = {p.decode_idx, p.poc, p.cvs, p.output, p.irap, p.idr, p.slice_type, p.slice_qp,
                          p.W, p.H, p.width, p.height, p.crop_x, p.crop_y, p.bit_depth, p.bit_depth_c,
                          p.log2_ctb, p.constrained_intra, p.strong_intra, p.lf_across_tiles, p.cb_qp_off, p.cr_qp_off,
                          p.deblock_any, p.sao_any};
    std::copy(vals, vals + 24, m);
    for (size_t k = 0; k < p.ref_ids.size() && k < 16; ++k) ref_ids[i * 16 + k] = p.ref_ids[k];
    const uint8_t* mb = reinterpret_cast<const uint8_t*>(p.mvf.data());
    mvf.insert(mvf.end(), mb, mb + p.mvf.size() * sizeof(hevc::DecMv4));
    mvf_sub_off[i] = static_cast<int64_t>(mvf_sub.size() / sizeof(hevc::DecMv4));
    const uint8_t* ms = reinterpret_cast<const uint8_t*>(p.mvf_sub.data());
    mvf_sub.insert(mvf_sub.end(), ms, ms + p.mvf_sub.size() * sizeof(hevc::DecMv4));
    bs.insert(bs.end(), p.bs.begin(), p.bs.end());
    const uint8_t* cb = reinterpret_cast<const uint8_t*>(p.ctbs.data());
    ctbs.insert(ctbs.end(), cb, cb + p.ctbs.size() * sizeof(hevc::DecCtb));
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(p.sao.data());
    sao.insert(sao.end(), sb, sb + p.sao.size() * sizeof(hevc::DecSao));
    if (!p.scaling.empty()) {
      if (scaling.empty()) scaling.assign(P * hevc::kScalingBytes, 16);
      std::memcpy(scaling.data() + i * hevc::kScalingBytes, p.scaling.data(), hevc::kScalingBytes);
    }
    tu_off[i] = static_cast<int64_t>(tus.size());
    op_off[i] = static_cast<int64_t>(ops.size());
    ref_off[i] = static_cast<int64_t>(refs.size());
    slice_off[i] = static_cast<int64_t>(slices.size());
    coef_off[i] = static_cast<int64_t>(coefs.size());
    tus.insert(tus.end(), p.tus.begin(), p.tus.end());
    ops.insert(ops.end(), p.ops.begin(), p.ops.end());
    refs.insert(refs.end(), p.refs.begin(), p.refs.end());
    slices.insert(slices.end(), p.slices.begin(), p.slices.end());
    coefs.insert(coefs.end(), p.coefs.begin(), p.coefs.end());
    std::copy(p.ops_off.begin(), p.ops_off.end(), ctb_ops.begin() + i * (nctb + 1));
    // the records are consumed: free them as we go (segments can be large)
    std::vector<hevc::DecMv4>().swap(p.mvf);
    std::vector<int16_t>().swap(p.coefs);
  }
  tu_off[P] = static_cast<int64_t>(tus.size());
  op_off[P] = static_cast<int64_t>(ops.size());
  ref_off[P] = static_cast<int64_t>(refs.size());
  slice_off[P] = static_cast<int64_t>(slices.size());
  coef_off[P] = static_cast<int64_t>(coefs.size());
  const py::ssize_t Pn = static_cast<py::ssize_t>(P);
  d["n"] = static_cast<int>(P);
  d["meta"] = to_array(meta, {Pn, 24});
  d["ref_ids"] = to_array(ref_ids, {Pn, 16});
  d["display"] = to_array(display, {Pn});
  mvf_sub_off[P] = static_cast<int64_t>(mvf_sub.size() / sizeof(hevc::DecMv4));
  d["mvf"] = to_array(mvf, {Pn, h4 / 2, w4 / 2, 12});
  d["mvf_sub"] = to_array(mvf_sub, {static_cast<py::ssize_t>(mvf_sub.size() / 12), 12});
  d["mvf_sub_off"] = to_array(mvf_sub_off, {Pn + 1});
  d["bs"] = to_array(bs, {Pn, h4, w4});
  d["ctbs"] = to_array(ctbs, {Pn, nctb, 8});
  d["sao"] = to_array(sao, {Pn, nctb, 24});
  d["scaling"] = scaling.empty() ? py::array_t<uint8_t>(std::vector<py::ssize_t>{0}) : to_array(scaling, {Pn, hevc::kScalingBytes});
  d["tus"] = raw_rows(tus);
  d["ops"] = raw_rows(ops);
  d["refs"] = raw_rows(refs);
  d["slices"] = raw_rows(slices);
  d["coefs"] = to_array(coefs, {static_cast<py::ssize_t>(coefs.size())});
  d["ctb_ops"] = to_array(ctb_ops, {Pn, nctb + 1});
  d["tu_off"] = to_array(tu_off, {Pn + 1});
  d["op_off"] = to_array(op_off, {Pn + 1});
  d["ref_off"] = to_array(ref_off, {Pn + 1});
  d["slice_off"] = to_array(slice_off, {Pn + 1});
  d["coef_off"] = to_array(coef_off, {Pn + 1});
  return d;
}

}  // namespace

// HEVC frame parameters from a Python dict; a collocated picture's records ("col_cu",
// uint8 [nctb * 16, 16]) are kept alive in `keep` while the GIL is released
hevc::HevcFrameParams hevc_frame_from(const py::dict& fp, std::vector<py::array>& keep, size_t cu_bytes) {
  hevc::HevcFrameParams f;
  f.idr = dget<int>(fp, "idr", 1);
  f.poc = dget<int>(fp, "poc", 0);
  f.qp = dget<int>(fp, "qp", 30);
  f.slice_type = f.idr ? 2 : dget<int>(fp, "slice_type", 1);
  f.nal_ref = dget<int>(fp, "nal_ref", 1);
  f.ref_poc[0] = dget<int>(fp, "ref_poc0", -1);
  f.ref_poc[1] = dget<int>(fp, "ref_poc1", -1);
  // several active pictures per list: "refs0" / "refs1" = RefPicListX POCs (entry 0 = ref_pocX)
  for (int l = 0; l < 2; ++l) {
    const char* key = l ? "refs1" : "refs0";
    if (!fp.contains(key) || fp[key].is_none()) continue;
    const py::list r = fp[key].cast<py::list>();
    if (r.size() < 1 || r.size() > static_cast<size_t>(hevc::kMaxRefs)) throw std::runtime_error("refsX: 1..4 entries");
    f.num_ref[l] = static_cast<int>(r.size());
    for (size_t i = 0; i < r.size(); ++i) f.list_poc[l][i] = r[i].cast<int>();
    if (f.ref_poc[l] < 0) f.ref_poc[l] = f.list_poc[l][0];
    if (f.list_poc[l][0] != f.ref_poc[l]) throw std::runtime_error("refsX[0] != ref_pocX");
  }
  if (fp.contains("rps")) {  // [(poc, used), ...]
    const py::list l = fp["rps"].cast<py::list>();
    if (l.size() > 8) throw std::runtime_error("rps: at most 8 entries");
    f.n_rps = static_cast<int>(l.size());
    for (size_t i = 0; i < l.size(); ++i) {
      const py::tuple e = l[i].cast<py::tuple>();
      f.rps_poc[i] = e[0].cast<int>();
      f.rps_used[i] = static_cast<uint8_t>(e[1].cast<int>() ? 1 : 0);
    }
  }
  if (fp.contains("wp") && !fp["wp"].is_none()) {  // [w_y, o_y, w_cb, o_cb, w_cr, o_cr]
    const py::list l = fp["wp"].cast<py::list>();
    if (l.size() != 6) throw std::runtime_error("wp: 6 entries (weight, offset per component)");
    f.wp = 1;
    for (int c = 0; c < 3; ++c) {
      f.wp_w[c] = l[2 * c].cast<int>();
      f.wp_o[c] = l[2 * c + 1].cast<int>();
      if (f.wp_w[c] < -64 || f.wp_w[c] > 191 || f.wp_o[c] < -128 || f.wp_o[c] > 127)
        throw std::runtime_error("wp: weight in -64..191, offset in -128..127");
    }
  }
  if (fp.contains("col_poc")) {
    f.col.set = 1;
    f.col.poc = dget<int>(fp, "col_poc", 0);
    f.col.ref_poc[0] = dget<int>(fp, "col_ref_poc0", 0);
    f.col.ref_poc[1] = dget<int>(fp, "col_ref_poc1", 0);
    for (int l = 0; l < 2; ++l) {  // "col_refs0" / "col_refs1": the col picture's list POCs
      for (int i = 0; i < hevc::kMaxRefs; ++i) f.col.list_poc[l][i] = f.col.ref_poc[l];
      const char* key = l ? "col_refs1" : "col_refs0";
      if (!fp.contains(key) || fp[key].is_none()) continue;
      const py::list r = fp[key].cast<py::list>();
      if (r.size() > static_cast<size_t>(hevc::kMaxRefs)) throw std::runtime_error("col_refsX: at most 4 entries");
      for (size_t i = 0; i < r.size(); ++i) f.col.list_poc[l][i] = r[i].cast<int>();
    }
    if (fp.contains("col_cu") && !fp["col_cu"].is_none()) {
      auto a = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>::ensure(fp["col_cu"]);
      if (!a || static_cast<size_t>(a.size()) != cu_bytes) throw std::runtime_error("col_cu: wrong size");
      keep.push_back(a);
      f.col.cu = reinterpret_cast<const hevc::CuInfo*>(a.data());
    }
  }
  return f;
}

PYBIND11_MODULE(_host, m) {
  m.doc() = "govideocompressor_amd host native library (bitstream, CAVLC, decoder, CPU encoder)";

  m.def("exp_golomb", [](const std::vector<int64_t>& vals, bool signed_) {
    BitWriter bw;
    for (int64_t v : vals) {
      if (signed_) bw.put_se(static_cast<int32_t>(v)); else bw.put_ue(static_cast<uint32_t>(v));
    }
    size_t bits = bw.bit_pos();
    bw.align_zero();
    return py::make_tuple(to_bytes(bw.bytes()), bits);
  });
  m.def("read_exp_golomb", [](py::bytes data, int count, bool signed_) {
    std::string s = data;
    BitReader br(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    std::vector<int64_t> out;
    for (int i = 0; i < count; ++i) out.push_back(signed_ ? br.get_se() : static_cast<int64_t>(br.get_ue()));
    return out;
  });
  m.def("cavlc_block", [](const std::vector<int>& coef, int start, int end, int max_num, int nc) {
    std::vector<int16_t> c(16, 0);
    for (size_t i = 0; i < coef.size() && i < 16; ++i) c[i] = static_cast<int16_t>(coef[i]);
    BitWriter bw;
    int tc = cavlc_write_block(bw, c.data(), start, end, max_num, nc);
    size_t bits = bw.bit_pos();
    bw.align_zero();
    return py::make_tuple(to_bytes(bw.bytes()), bits, tc);
  });
  m.def("table", [](const std::string& name) {
    std::vector<std::vector<int>> out;
    auto row = [&](const uint8_t* p, int n) { out.emplace_back(p, p + n); };
    if (name == "coeff_token_len") for (int t = 0; t < 4; ++t) row(kCoeffTokenLen[t], 68);
    else if (name == "coeff_token_bits") for (int t = 0; t < 4; ++t) row(kCoeffTokenBits[t], 68);
    else if (name == "chroma_dc_coeff_token") { row(kChromaDcCoeffTokenLen, 20); row(kChromaDcCoeffTokenBits, 20); }
    else if (name == "total_zeros_len") for (int t = 0; t < 15; ++t) row(kTotalZerosLen[t], 16);
    else if (name == "total_zeros_bits") for (int t = 0; t < 15; ++t) row(kTotalZerosBits[t], 16);
    else if (name == "chroma_dc_total_zeros_len") for (int t = 0; t < 3; ++t) row(kChromaDcTotalZerosLen[t], 4);
    else if (name == "chroma_dc_total_zeros_bits") for (int t = 0; t < 3; ++t) row(kChromaDcTotalZerosBits[t], 4);
    else if (name == "run_before_len") for (int t = 0; t < 7; ++t) row(kRunBeforeLen[t], 15);
    else if (name == "run_before_bits") for (int t = 0; t < 7; ++t) row(kRunBeforeBits[t], 15);
    else if (name == "intra_cbp") row(kGolombToIntraCbp, 48);
    else if (name == "inter_cbp") row(kGolombToInterCbp, 48);
    else if (name == "zigzag") row(kZigzag4x4, 16);
    else if (name == "lambda") out.emplace_back(kLambda, kLambda + 52);
    else if (name == "hevc_dct32") {
      for (int k = 0; k < 32; ++k) {
        std::vector<int> r(32);
        for (int n = 0; n < 32; ++n) r[n] = hevc::dct_coef(k, n);
        out.push_back(r);
      }
    }
    else throw std::runtime_error("unknown table " + name);
    return out;
  });

  m.def("selftest_i4_taps", &mivc::selftest_i4_taps);

  m.def("parameter_sets", [](const py::dict& cfg) {
    EncoderConfig c = cfg_from(cfg);
    return to_bytes(write_parameter_sets(make_sps(c), make_pps(c)));
  });

  // Write one slice NAL from MB decision arrays (uint8 [N,64] headers, int16 [N,408] coefficients).
  m.def(
      "write_slice",
      [](const py::dict& cfg, const py::dict& fp, py::array_t<uint8_t, py::array::c_style> hdr,
         py::array_t<int16_t, py::array::c_style> coef) {
        EncoderConfig c = cfg_from(cfg);
        SPS sps = make_sps(c);
        PPS pps = make_pps(c);
        int nmb = sps.width_mbs * sps.height_mbs;
        if (hdr.size() != static_cast<py::ssize_t>(nmb * sizeof(MbHeader))) throw std::runtime_error("header array has wrong size");
        if (coef.size() != static_cast<py::ssize_t>(nmb) * kCoefPerMb) throw std::runtime_error("coef array has wrong size");
        SliceHeader sh = slice_header_from(c, sps, pps, fp);
        const int num = dget<int>(fp, "num_mbs", nmb - sh.first_mb);  // MBs of this slice
        if (sh.first_mb < 0 || num < 1 || sh.first_mb + num > nmb) throw std::runtime_error("write_slice: bad MB range");
        SliceStats st;
        std::vector<uint8_t> nal;
        {
          py::gil_scoped_release rel;
          const MbHeader* mh = reinterpret_cast<const MbHeader*>(hdr.data());
          nal = pps.entropy_coding_mode ? write_slice_nal_cabac(sps, pps, sh, mh, coef.data(), num, &st)
                                        : write_slice_nal(sps, pps, sh, mh, coef.data(), num, &st);
        }
        py::dict stats;
        stats["bits"] = st.bits;
        stats["skipped"] = st.skipped;
        stats["intra"] = st.intra;
        stats["coded_inter"] = st.coded_inter;
        return py::make_tuple(to_bytes(nal), stats);
      },
      py::arg("cfg"), py::arg("frame"), py::arg("hdr"), py::arg("coef"));

  // CABAC slice data two ways: the serial writer and the GPU's symbol decomposition
  m.def("cabac_slice_data_two_ways", [](const py::dict& cfg, const py::dict& fp, py::array_t<uint8_t, py::array::c_style> hdr,
                                         py::array_t<int16_t, py::array::c_style> coef) {
    EncoderConfig c = cfg_from(cfg);
    c.cabac = 1;
    SPS sps = make_sps(c);
    PPS pps = make_pps(c);
    int nmb = sps.width_mbs * sps.height_mbs;
    if (hdr.size() != static_cast<py::ssize_t>(nmb * sizeof(MbHeader))) throw std::runtime_error("header array has wrong size");
    if (coef.size() != static_cast<py::ssize_t>(nmb) * kCoefPerMb) throw std::runtime_error("coef array has wrong size");
    SliceHeader sh = slice_header_from(c, sps, pps, fp);
    const MbHeader* mh = reinterpret_cast<const MbHeader*>(hdr.data());
    std::vector<uint8_t> a = cabac_slice_data(sps, pps, sh, mh, coef.data(), nmb);
    int nsyms = 0;
    std::vector<uint8_t> b = cabac_slice_data_symbols(sps, pps, sh, mh, coef.data(), nmb, &nsyms);
    return py::make_tuple(to_bytes(a), to_bytes(b), nsyms);
  });

  m.def(
      "decode",
      [](py::bytes data, bool skip_deblock) {
        std::string s = data;
        Decoder dec;
        dec.set_skip_deblock(skip_deblock);
        {
          py::gil_scoped_release rel;
          dec.decode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
          dec.flush();
        }
        py::list out;
        for (const DecodedPicture& p : dec.out()) out.append(picture_to_dict(p));
        return out;
      },
      py::arg("data"), py::arg("skip_deblock") = false);

  m.def(
      "parse",
      [](const std::vector<py::bytes>& segments, int threads) {
        // entropy decode only (CAVLC -> MbHeader + packed levels), one thread per segment
        std::vector<std::string> in;
        for (const py::bytes& b : segments) in.emplace_back(b);
        std::vector<ParsedSegment> res;
        {
          py::gil_scoped_release rel;
          res = h264_parse_many(in, threads);
        }
        py::list out;
        for (ParsedSegment& r : res) out.append(segment_to_dict(r));
        return out;
      },
      py::arg("segments"), py::arg("threads") = 1);

  // parsed batch kept in C++ (models/h264_decode_gpu.py): info(i) for planning, layout / pack
  // of one picture step straight into a pinned host buffer
  py::class_<H264Batch>(m, "H264Batch")
      .def("__len__", [](const H264Batch& b) { return b.segs.size(); })
      .def("info", [](const H264Batch& b, int i) { return segment_info(b.segs.at(i)); })
      .def("segment", [](H264Batch& b, int i) { return segment_to_dict(b.segs.at(i)); })
      .def("layout",
           [](const H264Batch& b, int t, const std::vector<int>& slots, int nmb) {
             H264StepLayout L = b.layout(t, slots, nmb);
             py::dict d;
             d["hdr"] = L.hdr;
             d["mask"] = L.mask;
             d["off"] = L.off;
             d["bs"] = L.bs;
             d["wp"] = L.wp;
             d["coef"] = L.coef;
             d["sub"] = L.sub;
             d["total"] = L.total;
             return d;
           })
      .def("pack",
           [](const H264Batch& b, int t, const std::vector<int>& slots, int nmb, uintptr_t dst, size_t capacity,
              int threads) {
             H264StepLayout L = b.layout(t, slots, nmb);
             if (L.total > capacity) throw std::invalid_argument("H264Batch.pack: buffer too small");
             py::gil_scoped_release rel;
             b.pack(t, slots, nmb, reinterpret_cast<uint8_t*>(dst), threads);
           },
           py::arg("t"), py::arg("slots"), py::arg("nmb"), py::arg("dst"), py::arg("capacity"), py::arg("threads") = 4);
  m.def(
      "parse_batch",
      [](const std::vector<py::bytes>& segments, int threads) {
        std::vector<std::string> in;
        for (const py::bytes& b : segments) in.emplace_back(b);
        auto* batch = new H264Batch();
        {
          py::gil_scoped_release rel;
          batch->segs = h264_parse_many(in, threads);
        }
        return batch;
      },
      py::arg("segments"), py::arg("threads") = 1, py::return_value_policy::take_ownership);

  // ---------------------------------------------------------------- HEVC
  m.def("hevc_parameter_sets", [](const py::dict& cfg) { return to_bytes(hevc::hevc_parameter_sets(hevc_cfg_from(cfg))); });
  m.def(
      "hevc_write_slice",
      [](const py::dict& cfg, const py::dict& fp, py::array_t<uint8_t, py::array::c_style> ctu,
         py::array_t<uint8_t, py::array::c_style> cu, py::array_t<int16_t, py::array::c_style> cy,
         py::array_t<int16_t, py::array::c_style> cb, py::array_t<int16_t, py::array::c_style> cr) {
        hevc::HevcConfig c = hevc_cfg_from(cfg);
        const py::ssize_t nctu = static_cast<py::ssize_t>(c.wctb()) * c.hctb();
        std::vector<py::array> keep;
        const hevc::HevcFrameParams f = hevc_frame_from(fp, keep, static_cast<size_t>(nctu) * hevc::kCusPerCtb * hevc::kCuInfoBytes);
        const py::ssize_t W = c.coded_width(), H = c.coded_height();
        if (ctu.size() != nctu * 32) throw std::runtime_error("ctu records: wrong size");
        if (cu.size() != nctu * hevc::kCusPerCtb * hevc::kCuInfoBytes) throw std::runtime_error("cu records: wrong size");
        if (cy.size() != W * H || cb.size() != W * H / 4 || cr.size() != W * H / 4)
          throw std::runtime_error("coefficient planes: wrong size");
        hevc::HevcSliceStats st;
        std::vector<uint8_t> nal;
        {
          py::gil_scoped_release rel;
          nal = hevc::hevc_write_slice(c, f, reinterpret_cast<const hevc::CtuInfo*>(ctu.data()),
                                       reinterpret_cast<const hevc::CuInfo*>(cu.data()), cy.data(), cb.data(), cr.data(),
                                       &st);
        }
        py::dict stats;
        stats["bins"] = st.bins;
        stats["bytes"] = st.bytes;
        stats["intra_cus"] = st.intra_cus;
        stats["inter_cus"] = st.inter_cus;
        stats["skip_cus"] = st.skip_cus;
        stats["merge_cus"] = st.merge_cus;
        return py::make_tuple(to_bytes(nal), stats);
      },
      py::arg("cfg"), py::arg("frame"), py::arg("ctu"), py::arg("cu"), py::arg("coef_y"), py::arg("coef_cb"),
      py::arg("coef_cr"));
  m.def(
      "hevc_write_slice_packed",
      [](const py::dict& cfg, const py::dict& fp, py::array_t<uint8_t, py::array::c_style> ctu,
         py::array_t<uint8_t, py::array::c_style> cu, py::array_t<uint64_t, py::array::c_style> nzmap,
         py::array_t<uint32_t, py::array::c_style> ctb_off, py::array_t<int16_t, py::array::c_style> levels) {
        // levels in the GPU encoder's packed form (hevc::PackedLevels)
        hevc::HevcConfig c = hevc_cfg_from(cfg);
        const py::ssize_t nctu = static_cast<py::ssize_t>(c.wctb()) * c.hctb();
        std::vector<py::array> keep;
        const hevc::HevcFrameParams f = hevc_frame_from(fp, keep, static_cast<size_t>(nctu) * hevc::kCusPerCtb * hevc::kCuInfoBytes);
        if (ctu.size() != nctu * 32) throw std::runtime_error("ctu records: wrong size");
        if (cu.size() != nctu * hevc::kCusPerCtb * hevc::kCuInfoBytes) throw std::runtime_error("cu records: wrong size");
        if (nzmap.size() != nctu * 2 || ctb_off.size() != nctu) throw std::runtime_error("packed maps: wrong size");
        if (levels.size() % 16) throw std::runtime_error("packed levels: not whole 4x4 blocks");
        hevc::PackedLevels pk;
        pk.nzmap = nzmap.data();
        pk.ctb_off = ctb_off.data();
        pk.levels = levels.data();
        pk.nblocks = static_cast<size_t>(levels.size() / 16);
        hevc::HevcSliceStats st;
        std::vector<uint8_t> nal;
        {
          py::gil_scoped_release rel;
          nal = hevc::hevc_write_slice(c, f, reinterpret_cast<const hevc::CtuInfo*>(ctu.data()),
                                       reinterpret_cast<const hevc::CuInfo*>(cu.data()), nullptr, nullptr, nullptr, &st,
                                       &pk);
        }
        py::dict stats;
        stats["bins"] = st.bins;
        stats["bytes"] = st.bytes;
        return py::make_tuple(to_bytes(nal), stats);
      },
      py::arg("cfg"), py::arg("frame"), py::arg("ctu"), py::arg("cu"), py::arg("nzmap"), py::arg("ctb_off"),
      py::arg("levels"));
  m.def(
      "hevc_slice_substreams",
      [](const py::dict& cfg, const py::dict& fp, py::array_t<uint8_t, py::array::c_style> ctu,
         py::array_t<uint8_t, py::array::c_style> cu, py::array_t<int16_t, py::array::c_style> cy,
         py::array_t<int16_t, py::array::c_style> cb, py::array_t<int16_t, py::array::c_style> cr) {
        // the slice data substreams the host writer codes for a picture (one per CTU row with
        // WPP), for checking hevc_assemble_slices against hevc_write_slice
        hevc::HevcConfig c = hevc_cfg_from(cfg);
        const py::ssize_t nctu = static_cast<py::ssize_t>(c.wctb()) * c.hctb();
        std::vector<py::array> keep;
        const hevc::HevcFrameParams f = hevc_frame_from(fp, keep, static_cast<size_t>(nctu) * hevc::kCusPerCtb * hevc::kCuInfoBytes);
        const py::ssize_t W = c.coded_width(), H = c.coded_height();
        if (ctu.size() != nctu * 32 || cu.size() != nctu * hevc::kCusPerCtb * hevc::kCuInfoBytes ||
            cy.size() != W * H || cb.size() != W * H / 4 || cr.size() != W * H / 4)
          throw std::runtime_error("records / planes: wrong size");
        std::vector<std::vector<uint8_t>> subs;
        hevc::hevc_write_slice(c, f, reinterpret_cast<const hevc::CtuInfo*>(ctu.data()),
                               reinterpret_cast<const hevc::CuInfo*>(cu.data()), cy.data(), cb.data(), cr.data(), nullptr,
                               nullptr, &subs);
        py::list out;
        for (auto& v : subs) out.append(to_bytes(v));
        return out;
      },
      py::arg("cfg"), py::arg("frame"), py::arg("ctu"), py::arg("cu"), py::arg("coef_y"), py::arg("coef_cb"),
      py::arg("coef_cr"));
  m.def("hevc_coder_pic", [](const py::dict& cfg, const py::dict& fp) {
    // the GPU entropy kernel's view of a picture (hevc_ctu_coder.h CoderPic) as bytes
    const hevc::HevcConfig c = hevc_cfg_from(cfg);
    std::vector<py::array> keep;
    const hevc::HevcFrameParams f =
        hevc_frame_from(fp, keep, static_cast<size_t>(c.wctb()) * c.hctb() * hevc::kCusPerCtb * hevc::kCuInfoBytes);
    const hevc::CoderPic p = hevc::hevc_coder_pic(c, f);
    return py::bytes(reinterpret_cast<const char*>(&p), sizeof(p));
  });
  m.def(
      "hevc_assemble_slices",
      [](const py::dict& cfg, const py::list& frames, py::array_t<uint8_t, py::array::c_style> data,
         py::array_t<uint64_t, py::array::c_style> offs, py::array_t<uint32_t, py::array::c_style> sizes,
         py::array_t<int32_t, py::array::c_style> errs, int threads) {
        // slice NALs of B pictures whose substreams the GPU coded (kernels/hevc_entropy.hip):
        // substream r of picture b is data[offs[b * nsub + r] ..][: sizes[b * nsub + r]]
        const hevc::HevcConfig c = hevc_cfg_from(cfg);
        const py::ssize_t B = static_cast<py::ssize_t>(frames.size());
        const int nsub = c.wpp ? c.hctu() : 1;
        const py::ssize_t n = B * nsub;
        if (offs.size() < n + 1 || sizes.size() < n || errs.size() < n) throw std::runtime_error("substream tables: wrong size");
        const uint64_t* po = offs.data();
        const uint32_t* psz = sizes.data();
        for (py::ssize_t i = 0; i < n; ++i) {
          if (errs.data()[i] != 0)
            throw std::runtime_error("HEVC slice " + std::to_string(i / nsub) + ": " + hevc::coder_error_text(errs.data()[i]));
          if (po[i] + psz[i] > static_cast<uint64_t>(data.size())) throw std::runtime_error("substream outside the buffer");
        }
        std::vector<hevc::HevcFrameParams> fps(B);
        std::vector<py::array> keep;
        for (py::ssize_t b = 0; b < B; ++b) fps[b] = hevc_frame_from(frames[b].cast<py::dict>(), keep, 0);
        std::vector<std::vector<uint8_t>> nals(B);
        std::vector<std::string> msg(B);
        {
          py::gil_scoped_release rel;
          std::atomic<py::ssize_t> next{0};
          auto work = [&] {
            std::vector<const uint8_t*> ptr(nsub);
            for (py::ssize_t b = next++; b < B; b = next++) {
              try {
                for (int r = 0; r < nsub; ++r) ptr[r] = data.data() + po[b * nsub + r];
                nals[b] = hevc::hevc_assemble_slice(c, fps[b], ptr.data(), psz + b * nsub, nsub);
              } catch (const std::exception& e) {
                msg[b] = e.what();
              }
            }
          };
          const int nt = std::max(1, std::min<int>(threads, static_cast<int>(B)));
          std::vector<std::thread> pool;
          for (int t = 1; t < nt; ++t) pool.emplace_back(work);
          work();
          for (std::thread& th : pool) th.join();
        }
        py::list out;
        for (py::ssize_t b = 0; b < B; ++b) {
          if (!msg[b].empty()) throw std::runtime_error("HEVC slice " + std::to_string(b) + ": " + msg[b]);
          out.append(to_bytes(nals[b]));
        }
        return out;
      },
      py::arg("cfg"), py::arg("frames"), py::arg("data"), py::arg("offs"), py::arg("sizes"), py::arg("errs"),
      py::arg("threads") = 1);
  m.def(
      "hevc_write_slices_packed",
      [](const py::dict& cfg, const py::list& frames, py::array_t<uint8_t, py::array::c_style> ctu,
         py::array_t<uint8_t, py::array::c_style> cu, py::array_t<uint64_t, py::array::c_style> nzmap,
         py::array_t<uint32_t, py::array::c_style> ctb_off, py::array_t<int16_t, py::array::c_style> levels,
         int threads, bool with_stats) {
        // One picture per slot of a batch step ([B, ...] arrays, frames[b] = frame params),
        // coded by `threads` native threads with the GIL released for the whole batch (a
        // Python thread per picture would queue on the GIL after every slice).
        hevc::HevcConfig c = hevc_cfg_from(cfg);
        const py::ssize_t B = static_cast<py::ssize_t>(frames.size());
        const py::ssize_t nctu = static_cast<py::ssize_t>(c.wctb()) * c.hctb();
        if (ctu.ndim() != 3 || ctu.shape(0) < B || ctu.shape(1) != nctu || ctu.shape(2) != 32)
          throw std::runtime_error("ctu records: expected [B, nctb, 32]");
        if (cu.size() < B * nctu * hevc::kCusPerCtb * hevc::kCuInfoBytes) throw std::runtime_error("cu records: wrong size");
        if (nzmap.size() < B * nctu * 2 || ctb_off.size() < B * nctu) throw std::runtime_error("packed maps: wrong size");
        if (levels.ndim() != 2 || levels.shape(0) < B || levels.shape(1) % 16) throw std::runtime_error("packed levels: [B, 16 n]");
        std::vector<hevc::HevcFrameParams> fps(B);
        std::vector<py::array> keep;
        for (py::ssize_t b = 0; b < B; ++b)
          fps[b] = hevc_frame_from(frames[b].cast<py::dict>(), keep,
                                   static_cast<size_t>(nctu) * hevc::kCusPerCtb * hevc::kCuInfoBytes);
        const size_t per_lv = static_cast<size_t>(levels.shape(1));
        std::vector<std::vector<uint8_t>> nals(B);
        std::vector<hevc::HevcSliceStats> sts(B);
        std::vector<std::string> errs(B);
        {
          py::gil_scoped_release rel;
          std::atomic<py::ssize_t> next{0};
          auto work = [&] {
            for (py::ssize_t b = next++; b < B; b = next++) {
              try {
                hevc::PackedLevels pk;
                pk.nzmap = nzmap.data() + static_cast<size_t>(b) * nctu * 2;
                pk.ctb_off = ctb_off.data() + static_cast<size_t>(b) * nctu;
                pk.levels = levels.data() + static_cast<size_t>(b) * per_lv;
                pk.nblocks = per_lv / 16;
                nals[b] = hevc::hevc_write_slice(
                    c, fps[b], reinterpret_cast<const hevc::CtuInfo*>(ctu.data() + static_cast<size_t>(b) * nctu * 32),
                    reinterpret_cast<const hevc::CuInfo*>(cu.data() + static_cast<size_t>(b) * nctu * hevc::kCusPerCtb * hevc::kCuInfoBytes),
                    nullptr, nullptr, nullptr, with_stats ? &sts[b] : nullptr, &pk);
              } catch (const std::exception& e) {
                errs[b] = e.what();
              }
            }
          };
          const int nt = std::max(1, std::min<int>(threads, static_cast<int>(B)));
          std::vector<std::thread> pool;
          for (int t = 1; t < nt; ++t) pool.emplace_back(work);
          work();
          for (std::thread& th : pool) th.join();
        }
        for (py::ssize_t b = 0; b < B; ++b)
          if (!errs[b].empty()) throw std::runtime_error("HEVC slice " + std::to_string(b) + ": " + errs[b]);
        py::list out;
        for (py::ssize_t b = 0; b < B; ++b) {
          if (!with_stats) {
            out.append(to_bytes(nals[b]));
            continue;
          }
          py::dict st;
          st["bins"] = sts[b].bins;
          st["intra_cus"] = sts[b].intra_cus;
          st["inter_cus"] = sts[b].inter_cus;
          st["skip_cus"] = sts[b].skip_cus;
          st["merge_cus"] = sts[b].merge_cus;
          out.append(py::make_tuple(to_bytes(nals[b]), st));
        }
        return out;
      },
      py::arg("cfg"), py::arg("frames"), py::arg("ctu"), py::arg("cu"), py::arg("nzmap"), py::arg("ctb_off"),
      py::arg("levels"), py::arg("threads") = 1, py::arg("with_stats") = false);
  m.def(
      "hevc_decode",
      [](py::bytes data, bool skip_filters) {
        std::string s = data;
        hevc::HevcDecoder dec;
        dec.set_skip_loop_filters(skip_filters);
        {
          py::gil_scoped_release rel;
          dec.decode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
        }
        py::list out;
        for (const hevc::HevcPicture& p : dec.out()) out.append(hevc_picture_to_dict(p));
        return out;
      },
      py::arg("data"), py::arg("skip_filters") = false);


  // ---------------------------------------------------------------- general HEVC decoder (hevc_dec.h)
  m.def(
      "hevc_decode_full",
      [](py::bytes data, bool recon, bool skip_filters) {
        std::string s = data;
        hevc::DecodeOptions o;
        o.recon = recon;
        o.skip_filters = skip_filters;
        hevc::HevcStreamDecoder dec(o);
        {
          py::gil_scoped_release rel;
          dec.decode(reinterpret_cast<const uint8_t*>(s.data()), s.size());
        }
        const std::vector<int> order = dec.output_order();
        std::vector<int> display(dec.pictures().size(), -1);
        for (size_t i = 0; i < order.size(); ++i) display[order[i]] = static_cast<int>(i);
        py::list out;
        for (size_t i = 0; i < dec.pictures().size(); ++i) {
          py::dict d = dec_picture_to_dict(dec.pictures()[i], recon);
          d["display"] = display[i];
          out.append(d);
        }
        return out;
      },
      py::arg("data"), py::arg("recon") = true, py::arg("skip_filters") = false);
  // parsed HEVC batch kept in C++ (models/hevc_decode_gpu.py): info(i) for planning,
  // layout / pack of one picture step straight into a pinned host buffer
  py::class_<HevcBatch>(m, "HevcBatch")
      .def("__len__", [](const HevcBatch& b) { return b.segs.size(); })
      .def("info",
           [](const HevcBatch& b, int i) {
             const HevcParsed& sp = b.segs.at(i);
             py::dict d;
             if (!sp.error.empty()) {
               d["n"] = 0;
               d["error"] = sp.error;
               return d;
             }
             const std::vector<hevc::DecPicture>& pics = sp.dec->pictures();
             const size_t P = pics.size();
             const py::ssize_t Pn = static_cast<py::ssize_t>(P);
             std::vector<int32_t> meta(P * 24, 0), ref_ids(P * 16, -1), display(P, -1);
             for (size_t k = 0; k < sp.order.size(); ++k) display[sp.order[k]] = static_cast<int32_t>(k);
             for (size_t k = 0; k < P; ++k) {
               const hevc::DecPicture& q = pics[k];
               const int v[24] = {q.decode_idx, q.poc, q.cvs, q.output, q.irap, q.idr, q.slice_type, q.slice_qp,
                                  q.W, q.H, q.width, q.height, q.crop_x, q.crop_y, q.bit_depth, q.bit_depth_c,
                                  q.log2_ctb, q.constrained_intra, q.strong_intra, q.lf_across_tiles, q.cb_qp_off,
                                  q.cr_qp_off, q.deblock_any, q.sao_any};
               std::copy(v, v + 24, &meta[k * 24]);
               for (size_t r = 0; r < q.ref_ids.size() && r < 16; ++r) ref_ids[k * 16 + r] = q.ref_ids[r];
             }
             d["n"] = static_cast<int>(P);
             d["error"] = py::none();
             d["meta"] = to_array(meta, {Pn, 24});
             d["ref_ids"] = to_array(ref_ids, {Pn, 16});
             d["display"] = to_array(display, {Pn});
             return d;
           })
      .def("layout",
           [](const HevcBatch& b, int t, const std::vector<int>& slots) {
             HevcStepLayout L = b.layout(t, slots);
             py::dict d;
             d["meta"] = L.meta;
             d["tu_base"] = L.tu_base;
             d["coef_base"] = L.coef_base;
             d["op_base"] = L.op_base;
             d["ref_base"] = L.ref_base;
             d["slice_base"] = L.slice_base;
             d["ctb_ops"] = L.ctb_ops;
             d["mvf"] = L.mvf;
             d["mvf_sub"] = L.mvf_sub;
             d["bs"] = L.bs;
             d["ctbs"] = L.ctbs;
             d["sao"] = L.sao;
             d["tus"] = L.tus;
             d["coefs"] = L.coefs;
             d["ops"] = L.ops;
             d["refs"] = L.refs;
             d["slices"] = L.slices;
             d["scaling"] = L.scaling;
             d["total"] = L.total;
             d["max_tus"] = L.max_tus;
             d["scaling_on"] = L.scaling_on;
             d["deblock_any"] = L.deblock_any;
             d["sao_any"] = L.sao_any;
             return d;
           })
      .def("pack",
           [](const HevcBatch& b, int t, const std::vector<int>& slots, uintptr_t dst, size_t capacity, int threads) {
             HevcStepLayout L = b.layout(t, slots);
             if (L.total > capacity) throw std::invalid_argument("HevcBatch.pack: buffer too small");
             py::gil_scoped_release rel;
             b.pack(t, slots, reinterpret_cast<uint8_t*>(dst), threads);
           },
           py::arg("t"), py::arg("slots"), py::arg("dst"), py::arg("capacity"), py::arg("threads") = 4);
  m.def(
      "hevc_parse_batch",
      [](const std::vector<py::bytes>& segments, int threads) {
        std::vector<std::string> in;
        for (const py::bytes& b : segments) in.emplace_back(b);
        auto* batch = new HevcBatch();
        {
          py::gil_scoped_release rel;
          batch->segs = hevc_parse_many(in, threads, false);
        }
        return batch;
      },
      py::arg("segments"), py::arg("threads") = 1, py::return_value_policy::take_ownership);
  m.def(
      "hevc_parse",
      [](const std::vector<py::bytes>& segments, int threads, bool recon) {
        // entropy decode + motion derivation of many segments, one thread per segment; the
        // GPU records of every segment (recon: also the CPU reconstruction, for tests)
        std::vector<std::string> in;
        for (const py::bytes& b : segments) in.emplace_back(b);
        std::vector<std::unique_ptr<hevc::HevcStreamDecoder>> decs(in.size());
        std::vector<std::string> err(in.size());
        {
          py::gil_scoped_release rel;
          std::atomic<size_t> next{0};
          int nt = std::max(1, std::min<int>(threads, static_cast<int>(in.size())));
          std::vector<std::thread> pool;
          for (int t = 0; t < nt; ++t)
            pool.emplace_back([&] {
              for (size_t i = next++; i < in.size(); i = next++) {
                hevc::DecodeOptions o;
                o.recon = recon;
                o.gpu_records = true;
                decs[i].reset(new hevc::HevcStreamDecoder(o));
                try {
                  decs[i]->decode(reinterpret_cast<const uint8_t*>(in[i].data()), in[i].size());
                } catch (const std::exception& e) {
                  err[i] = e.what();
                }
              }
            });
          for (std::thread& th : pool) th.join();
        }
        py::list out;
        for (size_t i = 0; i < in.size(); ++i) {
          py::dict d;
          if (!err[i].empty()) {
            d["n"] = 0;
            d["error"] = err[i];
          } else {
            const std::vector<int> order = decs[i]->output_order();
            d = dec_segment_records(decs[i]->pictures(), order);
            if (recon) {
              py::list pl;
              for (const hevc::DecPicture& p : decs[i]->pictures()) pl.append(dec_picture_to_dict(p, true));
              d["pictures"] = pl;
            }
          }
          decs[i].reset();
          out.append(d);
        }
        return out;
      },
      py::arg("segments"), py::arg("threads") = 1, py::arg("recon") = false);
  m.def("hevc_exercise", [](uint32_t seed) { return to_bytes(hevc::hevc_exercise(seed)); }, py::arg("seed"));
  m.def("hevc_stream_info", [](py::bytes data) {
    std::string s = data;
    const hevc::HevcStreamInfo si = hevc::hevc_stream_info(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    py::dict d;
    d["width"] = si.width;
    d["height"] = si.height;
    d["bit_depth"] = si.bit_depth;
    d["fps"] = si.fps;
    d["frames"] = si.pictures;
    d["irap_frames"] = si.irap;
    return d;
  });
  m.def(
      "hevc_split_pieces",
      [](py::bytes data, int min_frames) {
        std::string s = data;
        std::vector<std::vector<uint8_t>> parts;
        {
          py::gil_scoped_release rel;
          parts = hevc::hevc_split_pieces(reinterpret_cast<const uint8_t*>(s.data()), s.size(), min_frames);
        }
        py::list out;
        for (const auto& p : parts) out.append(to_bytes(p));
        return out;
      },
      py::arg("data"), py::arg("min_frames") = 1);

  py::class_<CpuEncoder>(m, "CpuEncoder")
      .def(py::init([](const py::dict& cfg) { return new CpuEncoder(cfg_from(cfg)); }))
      .def("encode",
           [](CpuEncoder& e, py::array_t<uint8_t, py::array::c_style> frames, int nframes, int idr_pic_id) {
             std::vector<uint8_t> out;
             {
               py::gil_scoped_release rel;
               out = e.encode(frames.data(), nframes, idr_pic_id);
             }
             return to_bytes(out);
           })
      .def("stats",
           [](CpuEncoder& e) {
             py::list l;
             for (const FrameStats& s : e.stats()) {
               py::dict d;
               d["type"] = s.type;
               d["qp"] = s.qp;
               d["bytes"] = s.bytes;
               d["psnr_y"] = s.psnr_y;
               l.append(d);
             }
             return l;
           })
      .def("recon_unfiltered",
           [](CpuEncoder& e) {
             const std::vector<uint8_t>& r = e.recon_unfiltered();
             py::array_t<uint8_t> a(static_cast<py::ssize_t>(r.size()));
             std::memcpy(a.mutable_data(), r.data(), r.size());
             return a;
           })
      .def("recon", [](CpuEncoder& e) {
        const std::vector<uint8_t>& r = e.recon();
        py::array_t<uint8_t> a(static_cast<py::ssize_t>(r.size()));
        std::memcpy(a.mutable_data(), r.data(), r.size());
        return a;
      });

  // Slice header as big-endian bit-order words (for the GPU CAVLC kernels) + bit count.
  m.def("slice_header_bits", [](const py::dict& cfg, const py::dict& fp) {
    EncoderConfig c = cfg_from(cfg);
    SPS sps = make_sps(c);
    PPS pps = make_pps(c);
    SliceHeader sh = slice_header_from(c, sps, pps, fp);
    BitWriter bw;
    write_slice_header(bw, sh, sps, pps);
    if (pps.entropy_coding_mode)
      while (!bw.byte_aligned()) bw.put_bit(1);  // cabac_alignment_one_bit: slice data starts byte-aligned
    size_t nbits = bw.bit_pos();
    bw.align_zero();
    std::vector<uint32_t> words((bw.bytes().size() + 3) / 4, 0);
    for (size_t i = 0; i < bw.bytes().size(); ++i) words[i / 4] |= static_cast<uint32_t>(bw.bytes()[i]) << (24 - 8 * (i % 4));
    return py::make_tuple(words, nbits);
  });
  // RBSP -> Annex-B NAL unit (start code, header byte, emulation prevention)
  m.def("nal_wrap", [](py::bytes rbsp, int nal_ref_idc, int nal_unit_type) {
    std::string s = rbsp;
    std::vector<uint8_t> v(s.begin(), s.end()), out;
    out.reserve(v.size() + v.size() / 64 + 8);
    append_nal(out, nal_ref_idc, nal_unit_type, v);
    return to_bytes(out);
  });
  // batched: one buffer of concatenated RBSPs + sizes -> list of NAL byte strings
  m.def("nal_wrap_many", [](py::array_t<uint8_t, py::array::c_style> buf, const std::vector<int64_t>& sizes,
                            int nal_ref_idc, int nal_unit_type, int align, const std::vector<int>& ref_idcs,
                            const std::vector<int>& unit_types) {
    // slice RBSPs back to back in buf, each starting at a multiple of `align` bytes; ref_idcs /
    // unit_types (optional): per-slice NAL header fields (slots coding different picture types)
    if (align < 1 || (align & (align - 1))) throw std::invalid_argument("nal_wrap_many: align must be a power of 2");
    if ((!ref_idcs.empty() && ref_idcs.size() != sizes.size()) || (!unit_types.empty() && unit_types.size() != sizes.size()))
      throw std::invalid_argument("nal_wrap_many: one nal_ref_idc / nal_unit_type per slice");
    int64_t need = 0;
    for (int64_t sz : sizes) {
      if (sz < 0) throw std::invalid_argument("nal_wrap_many: negative size");
      need = ((need + align - 1) & ~static_cast<int64_t>(align - 1)) + sz;
    }
    if (need > static_cast<int64_t>(buf.size())) throw std::invalid_argument("nal_wrap_many: sizes exceed the buffer");
    std::vector<std::vector<uint8_t>> outs(sizes.size());
    {
      py::gil_scoped_release rel;
      const uint8_t* p = buf.data();
      int64_t off = 0;
      for (size_t i = 0; i < sizes.size(); ++i) {
        off = (off + align - 1) & ~static_cast<int64_t>(align - 1);
        std::vector<uint8_t> v(p + off, p + off + sizes[i]);
        outs[i].reserve(v.size() + v.size() / 64 + 8);
        append_nal(outs[i], ref_idcs.empty() ? nal_ref_idc : ref_idcs[i], unit_types.empty() ? nal_unit_type : unit_types[i], v);
        off += sizes[i];
      }
    }
    py::list l;
    for (auto& o : outs) l.append(to_bytes(o));
    return l;
  }, py::arg("buf"), py::arg("sizes"), py::arg("nal_ref_idc"), py::arg("nal_unit_type"), py::arg("align") = 1,
     py::arg("ref_idcs") = std::vector<int>{}, py::arg("unit_types") = std::vector<int>{});

  m.def("parse_nals", [](py::bytes data) {
    std::string s = data;
    std::vector<NalUnit> v = parse_annexb(reinterpret_cast<const uint8_t*>(s.data()), s.size(), false);
    py::list l;
    for (const NalUnit& u : v) l.append(py::make_tuple(u.nal_unit_type, u.nal_ref_idc, u.offset, u.size));
    return l;
  });
  m.def("split_at_idr", [](py::bytes data, int min_frames) {
    std::string s = data;
    std::vector<std::pair<size_t, size_t>> cuts;
    {
      py::gil_scoped_release rel;
      cuts = split_annexb_at_idr(reinterpret_cast<const uint8_t*>(s.data()), s.size(), min_frames);
    }
    return cuts;
  });
  m.def("split_pieces", [](py::bytes data, int min_frames) {
    std::string s = data;
    std::vector<std::vector<uint8_t>> pieces;
    {
      py::gil_scoped_release rel;
      pieces = split_annexb_pieces(reinterpret_cast<const uint8_t*>(s.data()), s.size(), min_frames);
    }
    py::list l;
    for (auto& pc : pieces) l.append(to_bytes(pc));
    return l;
  });
  m.def("stream_info", [](py::bytes data) {
    std::string s = data;
    StreamInfo si = probe_annexb(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    py::dict d;
    d["width"] = si.width;
    d["height"] = si.height;
    d["fps"] = si.fps;
    d["frames"] = si.frames;
    d["idr_frames"] = si.idr_frames;
    d["profile_idc"] = si.profile_idc;
    d["level_idc"] = si.level_idc;
    d["entropy"] = si.cabac ? "cabac" : "cavlc";
    return d;
  });
  m.def("concat", [](const std::vector<py::bytes>& parts) {
    std::vector<std::string> ss;
    for (const py::bytes& b : parts) ss.push_back(b);
    std::vector<std::pair<const uint8_t*, size_t>> v;
    for (const std::string& s : ss) v.emplace_back(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    return to_bytes(concat_annexb(v));
  });
  m.def("mp4_mux", [](py::bytes data, double fps) {
    std::string s = data;
    return to_bytes(mux_mp4(reinterpret_cast<const uint8_t*>(s.data()), s.size(), fps));
  });
  m.def("h264_samples", [](py::bytes data) {
    std::string s = data;
    H264Samples hs;
    {
      py::gil_scoped_release rel;
      hs = h264_samples(reinterpret_cast<const uint8_t*>(s.data()), s.size());
    }
    py::dict d;
    d["data"] = to_bytes(hs.data);
    d["sizes"] = hs.sizes;
    d["sync"] = std::vector<int>(hs.sync.begin(), hs.sync.end());
    d["display"] = hs.display;
    d["sps"] = to_bytes(hs.sps);
    d["pps"] = to_bytes(hs.pps);
    d["width"] = hs.width;
    d["height"] = hs.height;
    d["fps"] = hs.fps;
    return d;
  });
  m.def("mp4_demux", [](py::bytes data) {
    std::string s = data;
    return to_bytes(demux_mp4_to_annexb(reinterpret_cast<const uint8_t*>(s.data()), s.size()));
  });
  m.def(
      "lowres_costs",
      [](py::array_t<uint8_t, py::array::c_style> frames, int width, int height, int nframes) {
        if (width < 2 || height < 2 || nframes < 0 || width % 2 || height % 2)
          throw std::invalid_argument("lowres_costs: bad geometry");
        if (static_cast<size_t>(frames.size()) < static_cast<size_t>(nframes) * width * height * 3 / 2)
          throw std::invalid_argument("lowres_costs: frame buffer smaller than nframes I420 frames");
        std::vector<float> intra(nframes), inter(nframes);
        {
          py::gil_scoped_release rel;
          lowres_frame_costs(frames.data(), width, height, nframes, intra.data(), inter.data());
        }
        return py::make_tuple(intra, inter);
      });
}
