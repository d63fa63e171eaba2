// gs_io.cpp -- base58, stake YAML and the synthetic network (see gs_io.h).
#include "gs_io.h"

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>

namespace gsio {

static const char* B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

std::string b58encode(const uint8_t* b, size_t n) {
  size_t zeros = 0;
  while (zeros < n && b[zeros] == 0) ++zeros;
  std::vector<uint8_t> digits;  // base-58 digits, least significant first
  for (size_t i = zeros; i < n; ++i) {
    uint32_t carry = b[i];
    for (auto& d : digits) {
      carry += (uint32_t)d << 8;
      d = (uint8_t)(carry % 58);
      carry /= 58;
    }
    while (carry) {
      digits.push_back((uint8_t)(carry % 58));
      carry /= 58;
    }
  }
  std::string s(zeros, '1');
  for (auto it = digits.rbegin(); it != digits.rend(); ++it) s.push_back(B58[*it]);
  return s;
}

bool b58decode_pubkey(const std::string& s, uint8_t out[32], std::string* why) {
  // solana-sdk Pubkey::from_str: len > MAX_BASE58_LEN (44) -> WrongSize; bs58 decode
  // failure -> Invalid; decoded length != 32 -> WrongSize.
  auto fail = [&](const char* m) {
    if (why) *why = m;
    return false;
  };
  if (s.size() > 44) return fail("WrongSize");
  size_t zeros = 0;
  while (zeros < s.size() && s[zeros] == '1') ++zeros;
  std::vector<uint8_t> bytes;  // little-endian
  for (size_t i = zeros; i < s.size(); ++i) {
    const char* p = std::strchr(B58, s[i]);
    if (!p || !*p) return fail("Invalid");
    uint32_t carry = (uint32_t)(p - B58);
    for (auto& x : bytes) {
      carry += (uint32_t)x * 58;
      x = (uint8_t)(carry & 0xFF);
      carry >>= 8;
    }
    while (carry) {
      bytes.push_back((uint8_t)(carry & 0xFF));
      carry >>= 8;
    }
  }
  if (zeros + bytes.size() != 32) return fail("WrongSize");
  std::memset(out, 0, 32);
  for (size_t i = 0; i < bytes.size(); ++i) out[31 - i] = bytes[i];
  return true;
}

static std::string trim(const std::string& x) {
  size_t a = 0, b = x.size();
  while (a < b && (x[a] == ' ' || x[a] == '\t' || x[a] == '\r')) ++a;
  while (b > a && (x[b - 1] == ' ' || x[b - 1] == '\t' || x[b - 1] == '\r')) --b;
  return x.substr(a, b - a);
}

bool read_stake_yaml(const std::string& path, std::vector<Account>& out, std::string& err) {
  std::ifstream f(path);
  if (!f) {
    err = "cannot open " + path + ": " + std::strerror(errno);
    return false;
  }
  out.clear();
  std::set<std::string> seen;
  std::string line;
  size_t ln = 0;
  while (std::getline(f, line)) {
    ++ln;
    std::string t = trim(line);
    if (t.empty() || t[0] == '#' || t == "---" || t == "..." || t == "{}") continue;
    std::string key, rest;
    if (t[0] == '\'' || t[0] == '"') {
      const char q = t[0];
      const size_t e = t.find(q, 1);
      if (e == std::string::npos) {
        err = path + ":" + std::to_string(ln) + ": unterminated quoted key";
        return false;
      }
      key = t.substr(1, e - 1);
      rest = trim(t.substr(e + 1));
      if (rest.empty() || rest[0] != ':') {
        err = path + ":" + std::to_string(ln) + ": expected ':' after key";
        return false;
      }
      rest = trim(rest.substr(1));
    } else {
      const size_t c = t.find(": ");
      if (c == std::string::npos) {
        err = path + ":" + std::to_string(ln) + ": expected `<pubkey>: <stake>`";
        return false;
      }
      key = trim(t.substr(0, c));
      rest = trim(t.substr(c + 2));
    }
    const size_t hash = rest.find(" #");
    if (hash != std::string::npos) rest = trim(rest.substr(0, hash));
    if (rest.empty() || rest.find_first_not_of("0123456789") != std::string::npos || rest.size() > 20) {
      err = path + ":" + std::to_string(ln) + ": stake is not a u64: " + rest;
      return false;
    }
    errno = 0;
    const unsigned long long v = std::strtoull(rest.c_str(), nullptr, 10);
    if (errno == ERANGE) {
      err = path + ":" + std::to_string(ln) + ": stake out of u64 range";
      return false;
    }
    if (!seen.insert(key).second) {
      err = path + ":" + std::to_string(ln) + ": duplicate key " + key;
      return false;
    }
    out.push_back({key, (uint64_t)v});
  }
  return true;
}

bool write_stake_yaml(const std::string& path, const std::vector<Account>& accts, std::string& err) {
  std::vector<Account> v = accts;
  std::sort(v.begin(), v.end(), [](const Account& a, const Account& b) { return a.key < b.key; });
  std::ofstream f(path);
  if (!f) {
    err = "cannot create " + path + ": " + std::strerror(errno);
    return false;
  }
  f << "---";
  for (auto& a : v) f << "\n" << a.key << ": " << a.stake;
  f << "\n";
  if (!f) {
    err = "write failed: " + path;
    return false;
  }
  return true;
}

// Philox4x32-10, the counter layout of the engine's streams (gs_device.h):
// key = seed halves, counter = {block, a, b, purpose}.
static void philox(uint32_t c[4], uint64_t seed) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t m0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t m1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(m1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(m0 >> 32) ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = (uint32_t)m1;
    c[2] = n2;
    c[3] = (uint32_t)m0;
  }
}

std::vector<Account> synthetic_network(uint32_t n) {
  std::vector<Account> v(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t c[4] = {0, i, 0, 0};
    philox(c, 0x5EED0001ull);
    const uint64_t jitter = ((uint64_t)c[0] | ((uint64_t)c[1] << 32)) % 1000000000ull;
    const uint64_t s = 15000000000000000ull / ((uint64_t)i + 1) + jitter;
    v[i].stake = std::max<uint64_t>(s, 1000000000ull);
    uint8_t pk[32];
    for (uint32_t blk = 0; blk < 2; ++blk) {
      uint32_t d[4] = {blk, i, 0, 0};
      philox(d, 0x5EED0002ull);
      for (int w = 0; w < 4; ++w)
        for (int k = 0; k < 4; ++k) pk[blk * 16 + w * 4 + k] = (uint8_t)(d[w] >> (8 * k));
    }
    v[i].key = b58encode(pk, 32);
  }
  return v;
}

std::vector<uint64_t> to_id_order(std::vector<Account>& accts) {
  std::sort(accts.begin(), accts.end(), [](const Account& a, const Account& b) { return a.key < b.key; });
  std::vector<uint64_t> st(accts.size());
  for (size_t i = 0; i < accts.size(); ++i) st[i] = accts[i].stake;
  return st;
}

}  // namespace gsio
