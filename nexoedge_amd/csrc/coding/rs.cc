// RSCode on MI355X.  Behaviour follows /root/reference/src/common/coding/rs.cc
// (line numbers cited per method); arithmetic runs in libnxec's gfx950
// kernels (nxec_encode_host / nxec_encode_host_ex), host code only plans.
#include "rs.hh"

#include "nxec_internal.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

extern "C" void nxec_cxx_abi_self(nxec_cxx_abi *out) {
  if (out) *out = RSCode::callerAbi();  // compiled here: libnxec's own layout
}

extern "C" int nxec_cxx_abi_check(const nxec_cxx_abi *c) {
  if (!c) return nxec::set_error(NXEC_ERR_INVALID, "nxec_cxx_abi_check: NULL layout");
  const nxec_cxx_abi s = RSCode::callerAbi();
  struct Field {
    const char *name;
    uint32_t nxec_cxx_abi::*m;
  };
  static const Field fields[] = {
      {"version", &nxec_cxx_abi::version},
      {"sizeof(Chunk)", &nxec_cxx_abi::size_chunk},
      {"alignof(Chunk)", &nxec_cxx_abi::align_chunk},
      {"offsetof(Chunk, fuuid)", &nxec_cxx_abi::off_chunk_uuid},
      {"offsetof(Chunk, chunkId)", &nxec_cxx_abi::off_chunk_id},
      {"offsetof(Chunk, data)", &nxec_cxx_abi::off_chunk_data},
      {"offsetof(Chunk, size)", &nxec_cxx_abi::off_chunk_size},
      {"offsetof(Chunk, freeData)", &nxec_cxx_abi::off_chunk_free},
      {"offsetof(Chunk, md5)", &nxec_cxx_abi::off_chunk_md5},
      {"offsetof(Chunk, digestData)", &nxec_cxx_abi::off_chunk_digest},
      {"sizeof(Chunk::fuuid)", &nxec_cxx_abi::size_uuid},
      {"sizeof(CodingOptions)", &nxec_cxx_abi::size_coding_options},
      {"sizeof(ByteBuffer)", &nxec_cxx_abi::size_byte_buffer},
      {"sizeof(DecodingPlan)", &nxec_cxx_abi::size_decoding_plan},
      {"sizeof(RSCode)", &nxec_cxx_abi::size_rscode},
  };
  for (const Field &f : fields)
    if (c->*f.m != s.*f.m)
      return nxec::set_error(NXEC_ERR_INVALID,
                             "C++ surface ABI mismatch: %s is %u in the caller, %u in libnxec (the caller's include "
                             "graph reached other Chunk/coding headers than libnxec's; see tools/overlay_reference.sh)",
                             f.name, c->*f.m, s.*f.m);
  return NXEC_OK;
}

// rs.cc:11-30, after the layout check (include/nxec.h §9)
RSCode::RSCode(CodingOptions options, const nxec_cxx_abi &callerLayout) {
  if (nxec_cxx_abi_check(&callerLayout) != NXEC_OK) throw std::invalid_argument(nxec_last_error());
  const coding_param_t n = options.getN(), k = options.getK();
  if (n <= 0 || k <= 0 || n < k) throw std::invalid_argument("RS codes only support n>=k, n > 0, and k > 0");
  _options = options;
  _name = "RS";
  nxec_gf_gen_rs_matrix(_encodeMatrix, n, k);  // rs.cc:26
}

num_t RSCode::getNumDataChunks() { return _options.getK(); }
num_t RSCode::getNumCodeChunks() { return _options.getN() - _options.getK(); }
num_t RSCode::getNumChunks() { return _options.getN(); }
num_t RSCode::getNumChunksPerNode() { return 1; }
length_t RSCode::getCodingStateSize() { return 0; }

// rs.cc:52-55: ceil(dataSize / k)
length_t RSCode::getChunkSize(length_t dataSize) {
  const coding_param_t k = _options.getK();
  return (dataSize + k - 1) / k;
}

// rs.cc:57-92: n chunks (32-B aligned), data chunks copied from `data`
// (caller zero-pads to k*chunkSize), parity computed on the GPU.
bool RSCode::encode(data_t *data, length_t dataSize, std::vector<Chunk> &stripe, data_t ** /*codingState*/) {
  const int k = _options.getK(), n = _options.getN();
  const length_t cs = getChunkSize(dataSize);
  stripe.clear();
  stripe.resize(n);
  std::vector<const unsigned char *> datap(k);
  std::vector<unsigned char *> codep(n - k > 0 ? n - k : 1);
  for (int i = 0; i < n; i++) {
    stripe.at(i).setChunkId(i);
    if (!stripe.at(i).allocateData(static_cast<int>(cs), /* aligned */ true)) {
      std::fprintf(stderr, "RSCode: failed to allocate chunk %d of %u bytes\n", i, cs);
      stripe.clear();
      return false;
    }
    if (i < k) datap[i] = stripe.at(i).data;
    else codep[i - k] = stripe.at(i).data;
  }
  // rs.cc:80's copy of the data into the chunks, spread over the library's
  // host pool (fresh chunk buffers fault their pages in on first touch)
  nxec::host_parallel_for(k, [&](int i) { std::memcpy(stripe[i].data, data + static_cast<size_t>(i) * cs, cs); });
  if (n == k || cs == 0) return true;
  // The caller hashes every chunk next (chunk_manager.cc:175): the GPU hashes
  // all n in the encode's own pass over the arena chunks (one lane's MD5
  // chain per chunk; the n chains run side by side), and each chunk carries
  // its digest to Chunk::computeMD5 (chunk.hh).  NXEC_CHUNK_MD5=0: no digests.
  const bool digests = nxec_chunk_md5_mode() >= 1;
  std::vector<unsigned char> md5(digests ? static_cast<size_t>(n) * 16 : 0);
  const int rc = digests ? nxec_encode_host_md5(static_cast<int>(cs), k, n - k, _encodeMatrix + k * k, datap.data(),
                                                codep.data(), md5.data(), md5.data() + 16 * k)
                         : nxec_encode_host(static_cast<int>(cs), k, n - k, _encodeMatrix + k * k, datap.data(),
                                            codep.data());
  if (rc != NXEC_OK) {
    std::fprintf(stderr, "RSCode::encode: %s\n", nxec_last_error());
    stripe.clear();
    return false;
  }
  if (digests)
    for (int i = 0; i < n; i++) {
      std::memcpy(stripe[i].md5, md5.data() + 16 * i, 16);
      stripe[i].setDigestValid();
    }
  return true;
}

// rs.cc:94-109: one partial -> copy; G partials -> XOR (all-ones 1 x G row)
bool RSCode::carRepairFinalize(unsigned char *inputp[], num_t numInputChunks, length_t chunkSize,
                               unsigned char *decodep[]) {
  if (numInputChunks == 1) {
    std::memcpy(decodep[0], inputp[0], chunkSize);
    return true;
  }
  std::vector<unsigned char> ones(numInputChunks, 1);
  return nxec_encode_host(static_cast<int>(chunkSize), static_cast<int>(numInputChunks), 1, ones.data(), inputp,
                          decodep) == NXEC_OK;
}

// rs.cc:111-236
bool RSCode::decode(std::vector<Chunk> &inputChunks, data_t **decodedData, length_t &decodedSize,
                    DecodingPlan & /*plan*/, data_t * /*codingState*/, bool isRepair,
                    std::vector<chunk_id_t> repairTargets) {
  const int k = _options.getK(), n = _options.getN();
  const num_t numInputs = static_cast<num_t>(inputChunks.size());
  const length_t cs = inputChunks.empty() ? 0 : static_cast<length_t>(inputChunks.at(0).size);
  const bool targetsGiven = !repairTargets.empty();

  if (numInputs < static_cast<num_t>(k) && (!isRepair || !_options.repairUsingCAR())) {  // rs.cc:134-137
    std::fprintf(stderr, "RSCode: insufficient input chunks (%u < %d)\n", numInputs, k);
    return false;
  }
  // inputs are matched to ids positionally and must be ascending (rs.cc:142-158)
  std::vector<int32_t> ids;
  for (int i = 0, idx = 0; i < n; i++) {
    if (idx < static_cast<int>(numInputs) && inputChunks.at(idx).chunkId == i) {
      ids.push_back(i);
      idx++;
    } else if (isRepair && !targetsGiven) {
      repairTargets.push_back(static_cast<chunk_id_t>(i));
    }
  }
  const num_t numDecoded = isRepair ? static_cast<num_t>(repairTargets.size()) : static_cast<num_t>(k);

  data_t *out = *decodedData;
  if (out == nullptr) {  // rs.cc:164-173
    out = static_cast<data_t *>(std::malloc(static_cast<size_t>(numDecoded) * cs + 1));
    if (!out) return false;
  }
  std::vector<unsigned char *> decodep(numDecoded > 0 ? numDecoded : 1);
  for (num_t i = 0; i < numDecoded; i++) decodep[i] = out + static_cast<size_t>(i) * cs;
  decodedSize = numDecoded * cs;
  std::vector<unsigned char *> inputp(numInputs > 0 ? numInputs : 1);
  for (num_t i = 0; i < numInputs; i++) inputp[i] = inputChunks.at(i).data;

  auto fail = [&]() {
    if (*decodedData != out) std::free(out);
    return false;
  };

  if (isRepair && numDecoded == 1 && _options.repairUsingCAR()) {  // rs.cc:184-192
    if (!carRepairFinalize(inputp.data(), numInputs, cs, decodep.data())) return fail();
    *decodedData = out;
    return true;
  }
  if (ids.size() < static_cast<size_t>(k)) return fail();
  if (cs == 0) {
    *decodedData = out;
    return true;
  }

  if (isRepair) {  // rs.cc:204-225: inverse rows for data targets, enc_row x inverse for parity targets
    std::vector<int32_t> tg(repairTargets.begin(), repairTargets.end());
    std::vector<unsigned char> m(static_cast<size_t>(tg.size()) * k + 1);
    if (nxec_rs_decode_matrix(n, k, ids.data(), tg.data(), static_cast<int>(tg.size()), m.data()) != NXEC_OK)
      return fail();
    // NXEC_CHUNK_MD5=2: the repaired chunks' digests from the same pass, for
    // the computeMD5 of each at chunk_manager.cc:1170-1173 (regions of *decodedData)
    const bool digests = nxec_chunk_md5_mode() >= 2 && !tg.empty();
    std::vector<unsigned char> md5(digests ? tg.size() * 16 : 0);
    if (digests) nxec_digest_clear();
    if ((digests ? nxec_encode_host_md5(static_cast<int>(cs), k, static_cast<int>(tg.size()), m.data(), inputp.data(),
                                        decodep.data(), nullptr, md5.data())
                 : nxec_encode_host(static_cast<int>(cs), k, static_cast<int>(tg.size()), m.data(), inputp.data(),
                                    decodep.data())) != NXEC_OK)
      return fail();
    for (size_t t = 0; digests && t < tg.size(); t++) nxec_digest_note(decodep[t], cs, md5.data() + 16 * t);
  } else {
    // all k data chunks (rs.cc:228-230 with the k x k inverse): the rows of
    // the inverse for erased data ids run on the GPU; the unit rows of the
    // surviving data ids are their input chunks, copied host to host by the
    // pool (routing them through the GPU pass cost 6 of 20 MiB of link
    // traffic per RS(10,4) 4-erasure call).
    std::vector<int32_t> tg;
    std::vector<int> src_of(k, -1);
    for (int j = 0; j < k; j++)
      if (ids[j] < k) src_of[ids[j]] = j;
    for (int d = 0; d < k; d++)
      if (src_of[d] < 0) tg.push_back(d);
    if (!tg.empty()) {
      std::vector<unsigned char> m(static_cast<size_t>(tg.size()) * k);
      if (nxec_rs_decode_matrix(n, k, ids.data(), tg.data(), static_cast<int>(tg.size()), m.data())) return fail();
      std::vector<unsigned char *> tp(tg.size());
      for (size_t t = 0; t < tg.size(); t++) tp[t] = decodep[tg[t]];
      if (nxec_encode_host(static_cast<int>(cs), k, static_cast<int>(tg.size()), m.data(), inputp.data(),
                           tp.data()) != NXEC_OK)
        return fail();
    }
    nxec::host_parallel_for(k, [&](int d) {
      if (src_of[d] >= 0 && decodep[d] != inputp[src_of[d]]) std::memcpy(decodep[d], inputp[src_of[d]], cs);
    });
  }
  *decodedData = out;
  return true;
}

// rs.cc:238-322
bool RSCode::preDecode(const std::vector<chunk_id_t> &failed, DecodingPlan &plan, data_t * /*codingState*/,
                       bool isRepair) {
  const int k = _options.getK(), n = _options.getN();
  const int nf = static_cast<int>(failed.size());
  if (nf > n - k) return false;  // rs.cc:244-247
  plan.release();
  std::vector<int32_t> f(failed.begin(), failed.end()), inputs(n);
  std::vector<unsigned char> rm(static_cast<size_t>(nf > 0 ? nf : 1) * k);
  int ni = 0, mi = 0;
  if (nxec_rs_plan(n, k, f.data(), nf, isRepair ? 1 : 0, inputs.data(), &ni, &mi, rm.data()) != NXEC_OK) {
    plan.release();
    return false;
  }
  for (int i = 0; i < ni; i++) plan.addInputChunkId(static_cast<chunk_id_t>(inputs[i]));
  plan.setMinNumInputChunks(static_cast<num_t>(mi));
  if (isRepair) {
    if (!plan.allocateRepairMatrix(static_cast<length_t>(nf) * k)) {
      plan.release();
      return false;
    }
    if (nf > 0) std::memcpy(plan.getRepairMatrix(), rm.data(), static_cast<size_t>(nf) * k);
  }
  return true;
}

bool RSCode::encodeStripes(nxec_ctx_t *ctx, unsigned char *dStripes, int64_t chunkStride, int64_t stripeStride,
                           int64_t chunkSize, int64_t numStripes, void *stream) {
  return nxec_rs_encode_stripes(ctx, _options.getN(), _options.getK(), dStripes, chunkStride, stripeStride, chunkSize,
                                numStripes, stream) == NXEC_OK;
}

bool RSCode::recoverStripes(nxec_ctx_t *ctx, const std::vector<chunk_id_t> &failed, unsigned char *dStripes,
                            int64_t chunkStride, int64_t stripeStride, int64_t chunkSize, int64_t numStripes,
                            void *stream) {
  std::vector<int32_t> f(failed.begin(), failed.end());
  return nxec_rs_recover_stripes(ctx, _options.getN(), _options.getK(), f.data(), static_cast<int>(f.size()),
                                 dStripes, chunkStride, stripeStride, chunkSize, numStripes, stream) == NXEC_OK;
}
