// archive.h -- zero-copy view of a libtorch `torch::save(module)` archive.
//
// The reference ships every model part between data owners and the aggregator
// as the bytes of `torch::save(task.model_part_, s)` (network_layer.cpp:305-313)
// and decodes them with `torch::load` (aggregator.cpp:63-64, ~0.5 GiB/s).  The
// archive is a zip of STORED (uncompressed, 64-byte aligned) records:
//   <prefix>/data.pkl            pickled module tree (protocol 2)
//   <prefix>/data/<key>          raw little-endian tensor storages
//   <prefix>/code/__torch__/*.py class declarations: __parameters__ / __buffers__
// This reader maps the tensors in place (no copy) in `named_parameters()`
// order -- the order aggregator.cpp:72-88 iterates -- and can emit a copy of
// the archive with new parameter values and rewritten CRC-32s, which
// `torch::load` on the data owner accepts (data_owner.cpp:232-253).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace fahost {

struct ZipEntry {
    std::string name;
    uint64_t data_offset = 0;   // first byte of the stored data
    uint64_t size = 0;          // uncompressed size
    uint64_t comp_size = 0;     // bytes on disk (== size for stored records)
    uint16_t method = 0;        // 0 stored, 8 deflate (only non-tensor records may be deflated)
    uint32_t crc = 0;
    uint64_t cd_offset = 0;     // central-directory header of this entry
    uint64_t local_offset = 0;  // local header of this entry
    uint64_t desc_offset = 0;   // data descriptor after the data (0 if none)
};

struct TensorView {
    std::string name;           // dotted path, e.g. "0.conv1.weight"
    std::string storage_type;   // "FloatStorage", "BFloat16Storage", "LongStorage", ...
    size_t elem_size = 0;
    std::vector<int64_t> sizes, strides;
    int64_t storage_offset = 0; // elements
    int64_t numel = 0;
    bool contiguous = false;
    int record = -1;            // index into entries()
    const uint8_t* data = nullptr;  // first element (storage + offset) inside the archive bytes
};

class TorchArchive {
public:
    // Parses `bytes[0, size)`; the memory must outlive the object (views point into it).
    bool parse(const uint8_t* bytes, size_t size, std::string* err);

    const std::vector<ZipEntry>& entries() const { return entries_; }
    const std::vector<TensorView>& params() const { return params_; }   // named_parameters(true) order
    const std::vector<TensorView>& buffers() const { return buffers_; } // named_buffers(true) order
    int64_t param_numel() const;
    bool params_are_float() const;
    // Bytes per parameter element when every parameter is fp32 (4) or every one is bf16 (2); 0 when
    // they are mixed or of another type (the bucket dtype of a receipt).
    int param_elem_size() const;

    // Contiguous pieces of the parameter bucket, in order (one per contiguous param, fp32 or bf16
    // throughout): a gather list for fa_submit_gather.  False if some param is strided or the types mix.
    bool param_segments(std::vector<const void*>* ptrs, std::vector<size_t>* bytes) const;
    // Strided-safe copy of all parameters (as fp32) into dst[param_numel()].
    bool gather_params(float* dst, std::string* err) const;
    // The same for either bucket dtype: param_numel() * param_elem_size() bytes, in their own type.
    bool gather_param_bytes(uint8_t* dst, std::string* err) const;
    // with_params_into for either bucket dtype: src holds the values in the parameters' own type.
    bool with_param_bytes_into(const uint8_t* src, uint8_t* dst, std::string* err) const;
    // A copy of the archive bytes with every parameter replaced by src (fp32, named order) and
    // the CRC-32 of every rewritten record updated in its data descriptor and central directory.
    bool with_params(const float* src, std::string* out, std::string* err) const;
    // Same, written into dst[0, size()) (e.g. straight into an outgoing frame).
    bool with_params_into(const float* src, uint8_t* dst, std::string* err) const;
    // The same in two steps, for a producer that writes the values itself (e.g. a D2H copy straight
    // into the outgoing frame): layout_into copies everything but the parameter values into dst and
    // returns where each parameter's values go (named_parameters order; false when a parameter is
    // strided or the parameters are not all fp32 or all bf16); seal_params then recomputes the CRC-32
    // of the parameter records.
    bool layout_into(uint8_t* dst, std::vector<void*>* param_dsts, std::vector<size_t>* param_bytes,
                     std::string* err) const;
    void seal_params(uint8_t* dst) const;
    // The same with the CRC-32s given, one per parameter in named_parameters order (e.g. computed on the GPU
    // from the reduced bucket, fa_output_crc32); false -- nothing written -- unless every parameter fills
    // its record exactly (the record's bytes are the parameter's, so the given CRC is the record's).
    bool seal_params_with(uint8_t* dst, const uint32_t* crcs) const;
    size_t size() const { return size_; }
    // Parses that took their tensor views from the layout cache (an archive with the same structure, pickle
    // and code records as one parsed before: every receipt of a bucket), process-wide.
    static unsigned long long layout_cache_hits();

private:
    const uint8_t* base_ = nullptr;
    size_t size_ = 0;
    std::string prefix_;
    std::vector<ZipEntry> entries_;
    std::vector<TensorView> params_, buffers_;
};

uint32_t crc32(const uint8_t* p, size_t n, uint32_t crc = 0);  // PCLMULQDQ folding where the CPU has it
uint32_t crc32_table(const uint8_t* p, size_t n, uint32_t crc = 0);  // the portable slicing-by-8 form

}  // namespace fahost
