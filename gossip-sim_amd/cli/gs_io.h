// gs_io.h -- host-side input formats of the gossip-sim driver.
//
//  - base58 (Bitcoin alphabet) of 32-byte pubkeys, with Pubkey::from_str's checks
//    (solana-sdk: at most 44 characters, decodes to exactly 32 bytes);
//  - the stake YAML map the reference reads with serde_yaml 0.8.26
//    (gossip_main.rs:304-318: HashMap<String, u64>) and writes from
//    write_accounts_main.rs:119-123;
//  - the deterministic synthetic power-law network of SURVEY.md 8(d), which stands in
//    for the reference's RPC account pull (make_gossip_cluster_from_rpc).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace gsio {

struct Account {
  std::string key;  // base58 pubkey
  uint64_t stake;
};

std::string b58encode(const uint8_t* bytes, size_t n);
// Pubkey::from_str: false (with a reason) for a string that is not a 32-byte base58 key.
bool b58decode_pubkey(const std::string& s, uint8_t out[32], std::string* why = nullptr);

// serde_yaml map of `<pubkey>: <u64>` entries (plain, single- or double-quoted keys;
// `---` / `...` document markers, comments and blank lines ignored). Duplicate keys
// and values that are not u64 are errors.
bool read_stake_yaml(const std::string& path, std::vector<Account>& out, std::string& err);
// serde_yaml 0.8 output of a HashMap<String, u64>: "---" then one `key: value` per
// line. HashMap order is arbitrary in the reference; here keys are written sorted.
bool write_stake_yaml(const std::string& path, const std::vector<Account>& accts, std::string& err);

// Synthetic network: node i has stake floor(1.5e16 / (i + 1)) +
// (philox_u64(0x5EED0001, i) mod 1e9), floored at 1 SOL, and pubkey = 32 bytes of
// Philox(0x5EED0002, i) blocks 0 and 1. Returned in generation order.
std::vector<Account> synthetic_network(uint32_t n);

// The engine's node order: ids are ranks of the base58 strings. Sorts
// `accts` by key and returns the stakes in id order.
std::vector<uint64_t> to_id_order(std::vector<Account>& accts);

}  // namespace gsio
