// vds_ec_wire.cpp -- the byte formats on either side of the codec on the live
// upload path, host code:
//
//   websocket "upload" -> base64 body (websocket_api.cpp:141-155,
//   base64::to_bytes, encoding.cpp:181-247) -> server_api::upload_data
//   (server_api.cpp:12-30: data hash = SHA-256 of the body) -> save_temp
//   (dht_network_client.cpp:62-107: every replica written, hashed, and kept
//   in <root>/tmp/<base64 of its hash, '+' -> '#', '/' -> '_'>) -> the JSON
//   answer {"replicas":[...],"hash":...,"replica_size":...}
//   (websocket_api.cpp:467-485, serialised by json_writer.cpp).
//
// The arithmetic in between (encode + the SHA-256 of every replica and of the
// body) runs on the GPU: vds_ec_save_temp16_host (vds_ec_api.cpp).
#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/vds_ec.h"

namespace {

const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

// base64::from_bytes (encoding.cpp:138-174): standard alphabet, '=' padding.
std::string b64(const uint8_t *d, size_t len) {
  std::string s;
  s.reserve((len + 2) / 3 * 4);
  for (; len > 2; len -= 3, d += 3) {
    const uint32_t t = (uint32_t(d[0]) << 16) | (uint32_t(d[1]) << 8) | d[2];
    s += kB64[(t >> 18) & 63];
    s += kB64[(t >> 12) & 63];
    s += kB64[(t >> 6) & 63];
    s += kB64[t & 63];
  }
  if (len == 1) {
    const uint32_t t = uint32_t(d[0]) << 16;
    s += kB64[(t >> 18) & 63];
    s += kB64[(t >> 12) & 63];
    s += "==";
  } else if (len == 2) {
    const uint32_t t = (uint32_t(d[0]) << 16) | (uint32_t(d[1]) << 8);
    s += kB64[(t >> 18) & 63];
    s += kB64[(t >> 12) & 63];
    s += kB64[(t >> 6) & 63];
    s += '=';
  }
  return s;
}

int copy_out(const std::string &s, char *out, size_t cap, size_t *out_len) {
  if (out_len) *out_len = s.size();
  if (!out) return VDS_EC_OK;  // size query
  if (cap < s.size() + 1) return VDS_EC_EINVAL;
  std::memcpy(out, s.data(), s.size());
  out[s.size()] = 0;
  return VDS_EC_OK;
}

}  // namespace

extern "C" {

size_t vds_ec_base64_decoded_size(const char *in, size_t len) {
  if (!in || len % 4) return 0;
  size_t padding = 0;
  if (len > 0 && in[len - 1] == '=') {
    ++padding;
    if (len > 1 && in[len - 2] == '=') ++padding;
  }
  return len / 4 * 3 - padding;
}

// base64::to_bytes (encoding.cpp:181-247), quirks kept: the output length is
// (len/4)*3 minus the '=' among the LAST TWO characters; the first '=' met
// ends the decode (whatever follows it) and emits one or two bytes by that
// trailing count; a '=' when the string does not end in one is "Invalid
// Padding"; any other character outside the alphabet (bytes >= 0x80
// included) is "Non-Valid Character".  Bytes of the output the reference
// leaves unwritten on such an early '=' (uninitialised malloc memory there)
// are zero here.
int vds_ec_base64_decode(const char *in, size_t len, uint8_t *out, size_t *out_len) {
  if ((len && !in) || !out_len) return VDS_EC_EINVAL;
  if (len % 4) return VDS_EC_EB64_LENGTH;
  const size_t size = vds_ec_base64_decoded_size(in, len);
  size_t padding = len / 4 * 3 - size;
  if (size && !out) return VDS_EC_EINVAL;
  if (size) std::memset(out, 0, size);
  uint32_t temp = 0;
  size_t offset = 0;
  int quantum = 0;
  for (size_t i = 0; i < len; ++i) {
    const char ch = in[i];
    temp <<= 6;
    if (ch >= 'A' && ch <= 'Z') {
      temp |= uint32_t(ch - 'A');
    } else if (ch >= 'a' && ch <= 'z') {
      temp |= uint32_t(ch - 'a' + 26);
    } else if (ch >= '0' && ch <= '9') {
      temp |= uint32_t(ch - '0' + 52);
    } else if (ch == '+') {
      temp |= 62u;
    } else if (ch == '/') {
      temp |= 63u;
    } else if (ch == '=') {
      if (padding == 1) {
        out[offset++] = uint8_t(temp >> 16);
        out[offset] = uint8_t(temp >> 8);
      } else if (padding == 2) {
        out[offset] = uint8_t(temp >> 10);
      } else {
        return VDS_EC_EB64_PADDING;
      }
      *out_len = size;
      return VDS_EC_OK;
    } else {
      return VDS_EC_EB64_CHAR;
    }
    if (++quantum == 4) {
      out[offset++] = uint8_t(temp >> 16);
      out[offset++] = uint8_t(temp >> 8);
      out[offset++] = uint8_t(temp);
      quantum = 0;
    }
  }
  *out_len = size;
  return VDS_EC_OK;
}

int vds_ec_base64_encode(const uint8_t *in, size_t len, char *out, size_t cap, size_t *out_len) {
  if (len && !in) return VDS_EC_EINVAL;
  return copy_out(b64(in, len), out, cap, out_len);
}

// save_temp's tmp-file names (dht_network_client.cpp:91-95): base64 of the
// replica's SHA-256 with '+' -> '#' and '/' -> '_', unsplit (the storage
// paths of save_data split it, vds_ec_replica_paths).  count names of
// VDS_EC_NAME_BYTES (44 characters + NUL) each.
int vds_ec_tmp_names(const uint8_t *digests, uint32_t count, char *out) {
  if (count && (!digests || !out)) return VDS_EC_EINVAL;
  for (uint32_t i = 0; i < count; ++i) {
    std::string s = b64(digests + 32ull * i, 32);
    for (char &c : s) c = c == '+' ? '#' : c == '/' ? '_' : c;
    std::memcpy(out + (size_t)VDS_EC_NAME_BYTES * i, s.c_str(), s.size() + 1);
  }
  return VDS_EC_OK;
}

// The websocket answer to "upload": process_message's {"id": id} with the
// "result" object websocket_api::upload adds (websocket_api.cpp:120-121,
// 472-482), as json_writer writes it: no whitespace, every primitive a
// quoted string (json_primitive holds text, json_writer.cpp:20-41), numbers
// included (json_object::add_property(name, uint64_t) stores to_string).
int vds_ec_upload_response_json(int id, const uint8_t *replica_digests, uint32_t n, const uint8_t *data_digest,
                                 uint32_t replica_size, char *out, size_t cap, size_t *out_len) {
  if ((n && !replica_digests) || !data_digest) return VDS_EC_EINVAL;
  std::string s = "{\"id\":\"" + std::to_string((uint64_t)(int64_t)id) + "\",\"result\":{\"replicas\":[";
  for (uint32_t i = 0; i < n; ++i) {
    if (i) s += ',';
    s += '"' + b64(replica_digests + 32ull * i, 32) + '"';
  }
  s += "],\"hash\":\"" + b64(data_digest, 32) + "\",\"replica_size\":\"" + std::to_string((uint64_t)replica_size) +
       "\"}}";
  return copy_out(s, out, cap, out_len);
}

}  // extern "C"
