#include "cabac_writer.h"

#include <stdexcept>

#include "../common/h264_cabac.h"

namespace mivc {
namespace h264 {

std::vector<uint8_t> cabac_slice_data(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                      const int16_t* coef, int num_mbs, SliceStats* stats) {
  if (!pps.entropy_coding_mode) throw std::runtime_error("CABAC writer called with a CAVLC PPS");
  if (sh.cabac_init_idc != 0) throw std::runtime_error("CABAC writer codes cabac_init_idc 0 only");
  if (pps.constrained_intra_pred) throw std::runtime_error("CABAC writer: constrained intra prediction is CAVLC-only");
  const int nmb = sps.width_mbs * sps.height_mbs;
  if (sh.first_mb < 0 || num_mbs <= 0 || sh.first_mb + num_mbs > nmb) throw std::runtime_error("bad MB range");
  for (int a = sh.first_mb; a < sh.first_mb + num_mbs; ++a) {
    const int k = mbs[a].kind;
    if (k == MBK_IPCM) throw std::runtime_error("I_PCM records are not written by the CABAC writer");
    if (sh.slice_type == SLICE_I && !mbk_is_intra(k)) throw std::runtime_error("inter MB in an I slice");
    if (sh.slice_type == SLICE_P && mbk_is_b(k)) throw std::runtime_error("B MB in a P slice");
    if (sh.slice_type == SLICE_B && !mbk_is_intra(k) && !mbk_is_b(k)) throw std::runtime_error("P MB in a B slice");
    if (k == MBK_I8x8 && !pps.transform_8x8_mode) throw std::runtime_error("I8x8 MB without transform_8x8_mode");
  }
  CabacSliceInfo si{};
  si.slice_type = sh.slice_type;
  si.wmb = sps.width_mbs;
  si.hmb = sps.height_mbs;
  si.first_mb = sh.first_mb;
  si.num_ref[0] = sh.num_ref_idx_l0_active;
  si.num_ref[1] = sh.num_ref_idx_l1_active;
  si.t8x8_mode = pps.transform_8x8_mode;
  si.slice_qp = pps.pic_init_qp + sh.slice_qp_delta;
  std::vector<CabacNb> nb(static_cast<size_t>(nmb));
  std::vector<uint8_t> out(static_cast<size_t>(num_mbs) * 160 + 4096);
  uint8_t states[kCabacContexts];
  for (int attempt = 0; attempt < 2; ++attempt) {
    CabacBuf buf{out.data(), out.size(), 0, 0};
    CabacEncoder e;
    CabacSliceStats st{};
    cabac_write_slice_data(si, nb.data(), states, &buf, mbs, coef, num_mbs, &e, &st);
    if (e.bad) throw std::runtime_error("CABAC carry past the start of the slice");
    if (!buf.overflow) {
      out.resize(buf.n);
      if (stats) {
        stats->skipped = st.skipped;
        stats->intra = st.intra;
        stats->coded_inter = st.inter;
      }
      return out;
    }
    out.assign(buf.n + 64, 0);
  }
  throw std::runtime_error("CABAC output buffer overflow");
}

std::vector<uint8_t> cabac_slice_data_symbols(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                              const int16_t* coef, int num_mbs, int* nsyms) {
  const int nmb = sps.width_mbs * sps.height_mbs;
  CabacSliceInfo si{};
  si.slice_type = sh.slice_type;
  si.wmb = sps.width_mbs;
  si.hmb = sps.height_mbs;
  si.first_mb = sh.first_mb;
  si.num_ref[0] = sh.num_ref_idx_l0_active;
  si.num_ref[1] = sh.num_ref_idx_l1_active;
  si.t8x8_mode = pps.transform_8x8_mode;
  si.slice_qp = pps.pic_init_qp + sh.slice_qp_delta;
  std::vector<CabacNb> nb(static_cast<size_t>(nmb));
  std::vector<uint16_t> syms(static_cast<size_t>(num_mbs) * 20000 + 1024);
  std::vector<uint8_t> out(static_cast<size_t>(num_mbs) * 4000 + 4096);
  uint8_t states[kCabacContexts];
  CabacBuf buf{out.data(), out.size(), 0, 0};
  cabac_write_slice_data_symbols(si, nb.data(), states, &buf, mbs, coef, num_mbs, syms.data(), syms.size(), nsyms);
  if (buf.overflow) throw std::runtime_error("CABAC symbol path overflow");
  out.resize(buf.n);
  return out;
}

std::vector<uint8_t> write_slice_nal_cabac(const SPS& sps, const PPS& pps, const SliceHeader& sh, const MbHeader* mbs,
                                           const int16_t* coef, int num_mbs, SliceStats* stats) {
  BitWriter bw;
  write_slice_header(bw, sh, sps, pps);
  while (!bw.byte_aligned()) bw.put_bit(1);  // cabac_alignment_one_bit
  std::vector<uint8_t> data = cabac_slice_data(sps, pps, sh, mbs, coef, num_mbs, stats);
  bw.append_bytes(data.data(), data.size());
  std::vector<uint8_t> nal;
  nal.reserve(bw.bytes().size() + bw.bytes().size() / 64 + 16);
  append_nal(nal, sh.nal_ref_idc, sh.nal_unit_type, bw.bytes());
  if (stats) stats->bits = static_cast<int>(nal.size() * 8);
  return nal;
}

}  // namespace h264
}  // namespace mivc
