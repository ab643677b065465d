// model.cc -- implementation of the restated memo interfaces (model.hh).
#include "model.hh"

#include <openssl/evp.h>

#include <algorithm>
#include <cstdio>
#include <filesystem>
#include <cstdio>
#include <random>
#include <sstream>

namespace memo_host {

std::string Address::hex() const {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (auto b : value) {
    s += d[b >> 4];
    s += d[b & 15];
  }
  return s;
}

Address Address::random(uint8_t fl) {
  static std::mutex mu;
  static std::mt19937_64 rng(0x6D656D6F);
  std::lock_guard<std::mutex> g(mu);
  uint8_t v[32];
  for (int i = 0; i < 32; i += 8) {
    const uint64_t x = rng();
    std::memcpy(v + i, &x, 8);
  }
  return Address(v, fl, true);
}

// OpenSSL 3 resolves EVP_sha256() through the provider store, under a lock,
// at every EVP_DigestInit_ex: with 16 pool threads hashing small blocks that
// lock serialised the plugin.  The digest is fetched once, and each thread
// reuses its own context.
namespace {
const EVP_MD* sha256_md() {
  static EVP_MD* md = EVP_MD_fetch(nullptr, "SHA256", nullptr);
  return md;
}
struct MdCtx {
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  ~MdCtx() { EVP_MD_CTX_free(c); }
};
}  // namespace

std::array<uint8_t, 32> sha256(const void* a, size_t na, const void* b, size_t nb) {
  std::array<uint8_t, 32> out;
  thread_local MdCtx ctx;
  EVP_MD_CTX* c = ctx.c;
  unsigned len = 0;
  const EVP_MD* md = sha256_md();
  if (!c || !md || EVP_DigestInit_ex(c, md, nullptr) != 1 || EVP_DigestUpdate(c, a, na) != 1 ||
      (b && nb && EVP_DigestUpdate(c, b, nb) != 1) || EVP_DigestFinal_ex(c, out.data(), &len) != 1)
    throw Error("sha256 failed");
  return out;
}

// ------------------------------------------------------------ remove keys
namespace {
struct PKey {
  EVP_PKEY* k = nullptr;
  ~PKey() { EVP_PKEY_free(k); }
};
struct MdSignCtx {
  EVP_MD_CTX* c = EVP_MD_CTX_new();
  ~MdSignCtx() { EVP_MD_CTX_free(c); }
};
}  // namespace

KeyPair KeyPair::generate() {
  PKey p;
  EVP_PKEY_CTX* c = EVP_PKEY_CTX_new_id(EVP_PKEY_ED25519, nullptr);
  const bool ok = c && EVP_PKEY_keygen_init(c) == 1 && EVP_PKEY_keygen(c, &p.k) == 1;
  EVP_PKEY_CTX_free(c);
  if (!ok) throw Error("ed25519 key generation failed");
  KeyPair kp;
  size_t n = 32;
  kp.public_key.resize(32);
  kp.private_key.resize(32);
  if (EVP_PKEY_get_raw_public_key(p.k, kp.public_key.data(), &n) != 1 || n != 32) throw Error("ed25519 key");
  n = 32;
  if (EVP_PKEY_get_raw_private_key(p.k, kp.private_key.data(), &n) != 1 || n != 32) throw Error("ed25519 key");
  return kp;
}

Buffer KeyPair::sign(const uint8_t* msg, size_t n) const {
  PKey p;
  p.k = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, nullptr, private_key.data(), private_key.size());
  MdSignCtx c;
  Buffer sig(64);
  size_t len = sig.size();
  if (!p.k || !c.c || EVP_DigestSignInit(c.c, nullptr, nullptr, nullptr, p.k) != 1 ||
      EVP_DigestSign(c.c, sig.data(), &len, msg, n) != 1)
    throw Error("ed25519 signing failed");
  sig.resize(len);
  return sig;
}

bool verify_signature(const Buffer& public_key, const Buffer& signature, const uint8_t* msg,
                      size_t n) {
  PKey p;
  p.k = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, nullptr, public_key.data(), public_key.size());
  MdSignCtx c;
  return p.k && c.c && EVP_DigestVerifyInit(c.c, nullptr, nullptr, nullptr, p.k) == 1 &&
         EVP_DigestVerify(c.c, signature.data(), signature.size(), msg, n) == 1;
}

void OwnerDirectory::set(const Address& owner, OwnerAcl acl) {
  std::lock_guard<std::mutex> g(mu_);
  acl_[owner] = std::move(acl);
}

std::optional<OwnerAcl> OwnerDirectory::find(const Address& owner) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = acl_.find(owner);
  if (it == acl_.end()) return std::nullopt;
  return it->second;
}

void OwnerDirectory::set_group(const Buffer& group_key, std::vector<Buffer> public_keys) {
  std::lock_guard<std::mutex> g(mu_);
  groups_[group_key] = std::move(public_keys);
}

std::optional<std::vector<Buffer>> OwnerDirectory::group_public_keys(const Buffer& group_key) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = groups_.find(group_key);
  if (it == groups_.end()) return std::nullopt;
  return it->second;
}

RemoveSignature chb_sign_remove(const Address& chb, const KeyPair& keys) {
  RemoveSignature rs;
  rs.signature_key = keys.public_key;
  rs.signature = keys.sign(chb.value.data(), chb.value.size());
  return rs;
}

RemoveSignature chb_sign_remove_group(const Address& chb, const Buffer& group_key,
                                      const KeyPair& current, int version) {
  RemoveSignature rs = chb_sign_remove(chb, current);
  rs.group_key = group_key;
  rs.group_index = version - 1;
  return rs;
}

std::string chb_validate_remove(const Address& chb, const Address& owner,
                                const RemoveSignature& rs, const OwnerDirectory* dir) {
  if (!owner) return "";
  if (!rs.signature_key || !rs.signature) return "Missing field in signature";
  const Buffer& key = *rs.signature_key;
  if (!verify_signature(key, *rs.signature, chb.value.data(), chb.value.size()))
    return "Invalid signature";
  const std::optional<OwnerAcl> acl = dir ? dir->find(owner) : std::nullopt;
  if (!acl) return "";  // owner block not found: allowed, as CHB.cc:222-227
  if (acl->world_write || acl->owner_key == key) return "";
  if (!rs.group_key) {
    for (auto& w : acl->writers)
      if (w == key) return "";
    return "Key not found";
  }
  // CHB.cc:243-258: the group's ACL entry must grant write, and the signing
  // key must be the group's key of version group_index + 1
  auto ge = std::find_if(acl->groups.begin(), acl->groups.end(),
                         [&](const GroupAclEntry& e) { return e.group_key == *rs.group_key; });
  if (ge == acl->groups.end() || !ge->write || !rs.group_index || !dir) return "Key not found";
  const auto pubs = dir->group_public_keys(*rs.group_key);
  const int gi = *rs.group_index;
  if (pubs && gi >= 0 && gi < (int)pubs->size() && (*pubs)[gi] == key) return "";
  return "Key not found";
}

Address chb_address(const Buffer& data, const Address& owner, const Buffer& salt,
                    const Version& version) {
  // salt || owner (the owner only when set and version >= 0.4), then data
  Buffer saltowner(salt);
  if (owner && !(version < Version{0, 4, 0}))
    saltowner.insert(saltowner.end(), owner.value.begin(), owner.value.end());
  const auto h = sha256(saltowner.data(), saltowner.size(), data.data(), data.size());
  return Address(h.data(), flags::immutable_block, !(version < Version{0, 5, 0}));
}

Block make_chb(Buffer data, Buffer salt, Address owner, const Version& version) {
  Block b;
  if (version < Version{0, 4, 0}) owner = Address();  // CHB.cc:44-46
  b.address = chb_address(data, owner, salt, version);
  b.data = std::move(data);
  b.salt = std::move(salt);
  b.owner = owner;
  return b;
}

Block make_mutable(Address address, Buffer data, int version) {
  Block b;
  address.value[Address::flag_byte] = flags::mutable_block;
  b.address = address;
  b.data = std::move(data);
  b.is_mutable = true;
  b.version = version;
  return b;
}

bool chb_valid(const Address& address, const Buffer& salt, const Address& owner, const Buffer& data,
               const Version& version) {
  const Address want = chb_address(data, owner, salt, version);
  return std::memcmp(want.value.data(), address.value.data(), 31) == 0;
}

// ------------------------------------------------------------- counters
size_t Counter::slot() {
  static std::atomic<size_t> next{0};
  thread_local const size_t s = next.fetch_add(1, std::memory_order_relaxed) % kSlots;
  return s;
}

// ---------------------------------------------------------------- silo
void Silo::check_space(size_t n) const {
  if (capacity_ >= 0 && usage_.load() + (int64_t)n > capacity_)
    throw silo::InsufficientSpace("insufficient space");
}

int Silo::set(const Key& k, const Buffer& v, bool insert, bool update) {
  check_space(v.size());
  const int delta = _set(k, v, insert, update);
  usage_ += delta;
  return delta;
}

int Silo::set(const Key& k, Buffer&& v, bool insert, bool update) {
  check_space(v.size());
  const int delta = _set_moved(k, std::move(v), insert, update);
  usage_ += delta;
  return delta;
}

int Silo::set_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n, bool insert,
                     bool update) {
  check_space(n);
  const int delta = _set_shared(k, std::move(bytes), n, insert, update);
  usage_ += delta;
  return delta;
}

int Silo::_set_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n, bool insert,
                      bool update) {
  return _set_moved(k, Buffer(bytes.get(), bytes.get() + n), insert, update);
}

int Silo::erase(const Key& k) {
  const int delta = _erase(k);
  usage_ += delta;
  return delta;
}

bool Silo::_read(const Key& k, const ReadSink& sink) const {
  Buffer v;
  if (!_try_get(k, v)) return false;
  sink(v.data(), v.size());
  return true;
}

bool Silo::_read_prefix(const Key& k, size_t n, const ReadSink& sink) const {
  Buffer v;
  if (!_try_get_prefix(k, n, v)) return false;
  sink(v.data(), v.size());
  return true;
}

bool Silo::_try_get(const Key& k, Buffer& out) const {
  try {
    out = _get(k);
    return true;
  } catch (silo::MissingKey&) {
    return false;
  }
}

bool Silo::_try_get_prefix(const Key& k, size_t n, Buffer& out) const {
  if (!_try_get(k, out)) return false;
  if (out.size() > n) out.resize(n);
  return true;
}

bool Silo::_contains(const Key& k) const {
  Buffer tmp;
  return _try_get(k, tmp);
}

bool MemorySilo::_contains(const Key& k) const {
  Stripe& st = stripe(k);
  std::lock_guard<std::mutex> g(st.mu);
  return st.blocks.count(k) != 0;
}

MemorySilo::Value MemorySilo::find(const Key& k) const {
  Stripe& st = stripe(k);
  std::lock_guard<std::mutex> g(st.mu);
  auto it = st.blocks.find(k);
  return it == st.blocks.end() ? Value() : it->second;
}

bool MemorySilo::_try_get(const Key& k, Buffer& out) const {
  const Value v = find(k);
  if (!v.p) return false;
  out.assign(v.p.get(), v.p.get() + v.n);
  return true;
}

bool MemorySilo::_try_get_prefix(const Key& k, size_t n, Buffer& out) const {
  const Value v = find(k);
  if (!v.p) return false;
  out.assign(v.p.get(), v.p.get() + std::min(n, v.n));
  return true;
}

// The sink runs under the stripe's lock, which keeps the value alive: no
// reference count is taken (values framed in one run share one, and every
// reader's increment and decrement would meet on its line).  Sinks must not
// call back into the silo.
bool MemorySilo::_read(const Key& k, const ReadSink& sink) const {
  Stripe& st = stripe(k);
  std::lock_guard<std::mutex> g(st.mu);
  auto it = st.blocks.find(k);
  if (it == st.blocks.end()) return false;
  sink(it->second.p.get(), it->second.n);
  return true;
}

bool MemorySilo::_read_prefix(const Key& k, size_t n, const ReadSink& sink) const {
  Stripe& st = stripe(k);
  std::lock_guard<std::mutex> g(st.mu);
  auto it = st.blocks.find(k);
  if (it == st.blocks.end()) return false;
  sink(it->second.p.get(), std::min(n, it->second.n));
  return true;
}

Buffer MemorySilo::_get(const Key& k) const {
  const Value v = find(k);
  if (!v.p) throw silo::MissingKey("missing key " + k.hex());
  return Buffer(v.p.get(), v.p.get() + v.n);
}

namespace {
// The bytes of a whole buffer, sharing its ownership (aliasing constructor).
std::shared_ptr<const uint8_t> bytes_of(std::shared_ptr<const Buffer> b) {
  const uint8_t* p = b->data();
  return std::shared_ptr<const uint8_t>(std::move(b), p);
}
}  // namespace

int MemorySilo::_set(const Key& k, const Buffer& v, bool insert, bool update) {
  // the copy, outside the lock
  return put(k, Value{bytes_of(std::make_shared<const Buffer>(v)), v.size()}, insert, update);
}

int MemorySilo::_set_moved(const Key& k, Buffer&& v, bool insert, bool update) {
  const size_t n = v.size();
  return put(k, Value{bytes_of(std::make_shared<const Buffer>(std::move(v))), n}, insert, update);
}

int MemorySilo::_set_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n, bool insert,
                            bool update) {
  return put(k, Value{std::move(bytes), n}, insert, update);
}

int MemorySilo::put(const Key& k, Value nv, bool insert, bool update) {
  Value old;  // freed outside the lock
  const int size = (int)nv.n;
  Stripe& st = stripe(k);
  std::lock_guard<std::mutex> g(st.mu);
  auto it = st.blocks.find(k);
  if (it == st.blocks.end()) {
    if (!insert) throw silo::MissingKey("missing key " + k.hex());
    st.blocks.emplace(k, std::move(nv));
    return size;
  }
  if (!update) throw silo::Collision("key exists " + k.hex());
  const int delta = size - (int)it->second.n;
  old = std::move(it->second);
  it->second = std::move(nv);
  return delta;
}

int MemorySilo::_erase(const Key& k) {
  Value old;
  Stripe& st = stripe(k);
  std::lock_guard<std::mutex> g(st.mu);
  auto it = st.blocks.find(k);
  if (it == st.blocks.end()) throw silo::MissingKey("missing key " + k.hex());
  const int delta = -(int)it->second.n;
  old = std::move(it->second);
  st.blocks.erase(it);
  return delta;
}

std::vector<Key> MemorySilo::_list() {
  std::vector<Key> out;
  for (auto& st : st_) {
    std::lock_guard<std::mutex> g(st.mu);
    for (auto& kv : st.blocks) out.push_back(kv.first);
  }
  std::sort(out.begin(), out.end());  // a deterministic order
  return out;
}

// ------------------------------------------------------ filesystem silo
namespace {
namespace fs = std::filesystem;
std::string hex_of(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}
bool key_of(const std::string& name, Key& out) {
  if (name.size() != 64) return false;
  uint8_t v[32];
  for (int i = 0; i < 32; ++i) {
    auto nib = [](char c) -> int {
      return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : -1;
    };
    const int hi = nib(name[2 * i]), lo = nib(name[2 * i + 1]);
    if (hi < 0 || lo < 0) return false;
    v[i] = (uint8_t)(hi << 4 | lo);
  }
  out = Address(v, 0, false);
  return true;
}
}  // namespace

FilesystemSilo::FilesystemSilo(std::string root, int64_t capacity)
    : Silo(capacity), root_(std::move(root)) {
  fs::create_directories(root_);
  int64_t used = 0;
  for (auto& dir : fs::directory_iterator(root_))
    if (dir.is_directory())
      for (auto& f : fs::directory_iterator(dir.path())) {
        Key k;
        if (f.is_regular_file() && key_of(f.path().filename().string(), k)) used += (int64_t)f.file_size();
      }
  usage_ += used;
}

std::string FilesystemSilo::path(const Key& k, bool make_dir) const {
  const std::string dir = root_ + "/" + hex_of(k.value.data(), 1);
  if (make_dir) fs::create_directories(dir);
  return dir + "/" + hex_of(k.value.data(), 32);
}

bool FilesystemSilo::_try_get(const Key& k, Buffer& out) const {
  std::FILE* f = std::fopen(path(k, false).c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? (size_t)n : 0);
  const size_t got = n > 0 ? std::fread(out.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  if (got != out.size()) throw Error("filesystem silo: short read " + k.hex());
  return true;
}

bool FilesystemSilo::_try_get_prefix(const Key& k, size_t n, Buffer& out) const {
  std::FILE* f = std::fopen(path(k, false).c_str(), "rb");
  if (!f) return false;
  out.resize(n);
  out.resize(std::fread(out.data(), 1, n, f));
  std::fclose(f);
  return true;
}

Buffer FilesystemSilo::_get(const Key& k) const {
  Buffer out;
  if (!_try_get(k, out)) throw silo::MissingKey("missing key " + k.hex());
  return out;
}

bool FilesystemSilo::_contains(const Key& k) const { return fs::exists(path(k, false)); }

int FilesystemSilo::_set(const Key& k, const Buffer& v, bool insert, bool update) {
  const std::string p = path(k, true);
  std::lock_guard<std::mutex> g(mu_);
  std::error_code ec;
  const bool exists = fs::exists(p);
  const int64_t old = exists ? (int64_t)fs::file_size(p, ec) : 0;
  if (!exists && !insert) throw silo::MissingKey("missing key " + k.hex());
  if (exists && !update) throw silo::Collision("key exists " + k.hex());
  const std::string tmp = p + ".tmp";
  std::FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw Error("filesystem silo: cannot write " + tmp);
  const size_t put = v.empty() ? 0 : std::fwrite(v.data(), 1, v.size(), f);
  const bool ok = std::fclose(f) == 0 && put == v.size();
  if (!ok) {
    fs::remove(tmp, ec);
    throw Error("filesystem silo: short write " + k.hex());
  }
  fs::rename(tmp, p);
  return (int)((int64_t)v.size() - old);
}

int FilesystemSilo::_erase(const Key& k) {
  const std::string p = path(k, false);
  std::lock_guard<std::mutex> g(mu_);
  std::error_code ec;
  if (!fs::exists(p)) throw silo::MissingKey("missing key " + k.hex());
  const int64_t old = (int64_t)fs::file_size(p, ec);
  fs::remove(p);
  return -(int)old;
}

std::vector<Key> FilesystemSilo::_list() {
  std::vector<Key> out;
  for (auto& dir : fs::directory_iterator(root_))
    if (dir.is_directory())
      for (auto& f : fs::directory_iterator(dir.path())) {
        Key k;
        if (f.is_regular_file() && key_of(f.path().filename().string(), k)) out.push_back(k);
      }
  return out;
}

// ---------------------------------------------------------------- nodes
void Node::store(const Key& k, const Buffer& v) {
  if (!up || evicted) throw Unavailable("node down");
  if (fail_stores) throw Unavailable("store refused");
  local->validate(k, v.data(), v.size());
  silo->set(k, v, true, true);
  ++stores;
}

void Node::store(const Key& k, Buffer&& v) {
  if (!up || evicted) throw Unavailable("node down");
  if (fail_stores) throw Unavailable("store refused");
  local->validate(k, v.data(), v.size());
  silo->set(k, std::move(v), true, true);
  ++stores;
}

void Node::store_shared(const Key& k, std::shared_ptr<const uint8_t> bytes, size_t n) {
  if (!up || evicted) throw Unavailable("node down");
  if (fail_stores) throw Unavailable("store refused");
  local->validate(k, bytes.get(), n);
  silo->set_shared(k, std::move(bytes), n, true, true);
  ++stores;
}

bool Node::try_read(const Key& k, const ReadSink& sink) const {
  if (!up || evicted) throw Unavailable("node down");
  fetches++;
  return silo->read(k, sink);
}

Buffer Node::fetch(const Key& k) const {
  if (!up || evicted) throw Unavailable("node down");
  fetches++;
  return silo->get(k);
}

void Node::remove(const Key& k) {
  if (!up || evicted) throw Unavailable("node down");
  ++remove_requests;
  silo->erase(k);
}

int Node::remove_values(const std::vector<Key>& keys, size_t prefix, const RemoveCheck& check,
                        std::string* refused) {
  if (!up || evicted) throw Unavailable("node down");
  ++remove_requests;
  int n = 0;
  for (auto& k : keys) {
    Buffer head;
    if (!silo->try_get_prefix(k, prefix, head)) continue;  // not here
    std::string why = check(k, head);
    if (!why.empty()) {
      if (refused) *refused = std::move(why);
      continue;
    }
    try {
      silo->erase(k);
      ++n;
    } catch (silo::MissingKey&) {  // erased meanwhile
    }
  }
  return n;
}

bool Node::try_fetch(const Key& k, Buffer& out) const {
  if (!up || evicted) throw Unavailable("node down");
  fetches++;
  return silo->try_get(k, out);
}

bool Node::try_fetch_prefix(const Key& k, size_t n, Buffer& out) const {
  if (!up || evicted) throw Unavailable("node down");
  return silo->try_get_prefix(k, n, out);
}

bool Node::has(const Key& k) const { return silo->contains(k); }

bool Node::holds_any(const std::vector<Key>& keys) const {
  if (!up || evicted) throw Unavailable("node down");
  for (auto& k : keys)
    if (silo->contains(k)) return true;
  return false;
}

namespace {
// A handle that does not own the node (the overlay does): copying it touches
// no reference count.
std::shared_ptr<Node> handle(Node* n) { return n ? std::shared_ptr<Node>(std::shared_ptr<Node>(), n) : nullptr; }
}  // namespace

Overlay::Overlay() {
  snaps_.push_back(std::make_unique<Snapshot>());
  snap_.store(snaps_.back().get(), std::memory_order_release);
}

Overlay::~Overlay() = default;

// ----------------------------------------------------------------- peers
Local::Local(std::unique_ptr<Silo> storage, std::optional<int> port, std::optional<IpAddress> listen)
    : storage_(std::move(storage)), port_(port.value_or(0)), listen_(std::move(listen)) {
  if (!storage_) throw Error("local: no storage");
}

void Local::validate(const Key&, const uint8_t*, size_t) const {}

std::shared_ptr<Node> Overlay::add_node(const Address& id, std::unique_ptr<Silo> silo) {
  return add_node(id, std::make_unique<Local>(std::move(silo)));
}

std::shared_ptr<Node> Overlay::add_node(const Address& id, std::unique_ptr<Local> local) {
  auto n = std::make_shared<Node>();
  n->id = id;
  n->silo = &local->storage();
  n->local = std::move(local);
  {
    std::lock_guard<std::mutex> g(mu_);
    auto next = std::make_unique<Snapshot>(*snap());
    next->nodes.push_back(n.get());
    next->by_id[n->id] = n.get();
    owned_.push_back(n);
    snaps_.push_back(std::move(next));
    snap_.store(snaps_.back().get(), std::memory_order_release);
  }
  notify([](const Handlers& h) -> const NodeEvent& { return h.discovered; }, id);
  return n;
}

int Overlay::subscribe(Handlers h) {
  std::lock_guard<std::mutex> g(hmu_);
  handlers_[next_token_] = std::move(h);
  return next_token_++;
}

void Overlay::unsubscribe(int token) {
  std::lock_guard<std::mutex> g(hmu_);
  handlers_.erase(token);
}

void Overlay::set_up(const Address& id, bool up) {
  auto n = node(id);
  if (!n) throw Error("overlay: unknown node " + id.hex());
  if (n->up.exchange(up) == up) return;
  if (up) notify([](const Handlers& h) -> const NodeEvent& { return h.appeared; }, id);
  else notify([](const Handlers& h) -> const NodeEvent& { return h.disappeared; }, id);
}

std::shared_ptr<Node> Overlay::node(const Address& id) const {
  const Snapshot* s = snap();
  auto it = s->by_id.find(id);
  return it == s->by_id.end() ? nullptr : handle(it->second);
}

std::vector<std::shared_ptr<Node>> Overlay::nodes() const {
  const Snapshot* s = snap();
  std::vector<std::shared_ptr<Node>> out;
  out.reserve(s->nodes.size());
  for (Node* n : s->nodes) out.push_back(handle(n));
  return out;
}

size_t Overlay::size() const { return snap()->nodes.size(); }

namespace {
// Rendezvous score of (address, node): a 64-bit mix of both ids (the ids are
// already hashes; the ranking needs dispersion, not collision resistance).
uint64_t rendezvous(const Address& a, const Address& n) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int w = 0; w < 4; ++w) {
    uint64_t x, y;
    std::memcpy(&x, a.value.data() + 8 * w, 8);
    std::memcpy(&y, n.value.data() + 8 * w, 8);
    h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h ^= y * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 31)) * 0x94D049BB133111EBull;
  }
  return h ^ (h >> 29);
}
}  // namespace

std::vector<std::shared_ptr<Node>> Overlay::rank(const Address& address) const {
  const Snapshot* sn = snap();
  std::vector<std::pair<uint64_t, Node*>> scored;
  scored.reserve(sn->nodes.size());
  for (Node* n : sn->nodes) scored.push_back({rendezvous(address, n->id), n});
  std::sort(scored.begin(), scored.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<std::shared_ptr<Node>> out;
  out.reserve(scored.size());
  for (auto& s : scored) out.push_back(handle(s.second));
  return out;
}

std::vector<std::shared_ptr<Node>> Overlay::allocate(const Address& address, int n) const {
  std::vector<std::shared_ptr<Node>> out;
  for (auto& nd : rank(address)) {
    if ((int)out.size() == n) break;
    if (nd->up && !nd->evicted) out.push_back(nd);
  }
  return out;
}

std::vector<std::shared_ptr<Node>> Overlay::lookup(const Address& address, int n) const {
  std::vector<std::shared_ptr<Node>> out;
  for (auto& nd : rank(address)) {
    if ((int)out.size() == n) break;
    if (!nd->evicted) out.push_back(nd);
  }
  return out;
}

// ------------------------------------------------------------- consensus
void Consensus::_fetch(const std::vector<AddressVersion>& addresses, ReceiveBlock res) {
  for (auto& a : addresses) {
    std::unique_ptr<Block> b;
    try {
      b = fetch(a.first, a.second);
    } catch (Error&) {
      res(a.first, nullptr, std::current_exception());
      continue;
    }
    res(a.first, std::move(b), nullptr);
  }
}

std::unique_ptr<Consensus::Stat> Consensus::stat(const Address&) { return std::make_unique<Stat>(); }

std::unique_ptr<Local> Consensus::make_local(std::optional<int> port, std::optional<IpAddress> listen_address,
                                             std::unique_ptr<Silo> storage) {
  return std::make_unique<Local>(std::move(storage), port, std::move(listen_address));
}

std::shared_ptr<Remote> Consensus::make_remote(std::shared_ptr<DockConnection> connection) {
  return std::make_shared<Remote>(std::move(connection));
}

std::string Consensus::redundancy() { return to_json({{"desired_factor", "1.0"}, {"type", "none"}}); }

std::string Consensus::stats() { return to_json({{"type", "none"}}); }

// ----------------------------------------------------------- replication
namespace {
Key replica_key(const Address& a) { return a; }

Buffer encode_replica(const Block& b) {
  // [version u32][salt len u32][owner 32][salt][data]
  Buffer out(40 + b.salt.size() + b.data.size());
  const uint32_t v = (uint32_t)b.version, sl = (uint32_t)b.salt.size();
  std::memcpy(out.data(), &v, 4);
  std::memcpy(out.data() + 4, &sl, 4);
  std::memcpy(out.data() + 8, b.owner.value.data(), 32);
  std::copy(b.salt.begin(), b.salt.end(), out.begin() + 40);
  std::copy(b.data.begin(), b.data.end(), out.begin() + 40 + sl);
  return out;
}

// The fields of a replica value without copying its data.
struct ReplicaView {
  uint32_t version;
  Address owner;
  const uint8_t* salt;
  uint32_t salt_len;
  const uint8_t* data;
  size_t data_len;
};
ReplicaView view_replica(const uint8_t* r, size_t n) {
  if (n < 40) throw ValidationFailed("short replica");
  ReplicaView v;
  std::memcpy(&v.version, r, 4);
  std::memcpy(&v.salt_len, r + 4, 4);
  if (40 + (size_t)v.salt_len > n) throw ValidationFailed("bad replica");
  v.owner = Address(r + 8, 0, false);
  v.salt = r + 40;
  v.data = r + 40 + v.salt_len;
  v.data_len = n - 40 - v.salt_len;
  return v;
}

Block decode_replica(const Address& a, const uint8_t* r, size_t n) {
  const ReplicaView v = view_replica(r, n);
  Block b;
  b.address = a;
  b.version = (int)v.version;
  b.is_mutable = a.mutable_block();
  b.owner = v.owner;
  b.salt.assign(v.salt, v.salt + v.salt_len);
  b.data.assign(v.data, v.data + v.data_len);
  return b;
}

// Paxos::LocalPeer restated for the replication path: what it stores is
// validated as LocalPeer::store does (Paxos.cc:1568-1615).
class ReplicaLocal : public Local {
 public:
  using Local::Local;
  void validate(const Key& k, const uint8_t* v, size_t n) const override {
    validate_replica(k, v, n);
    // validate with the previous version, if any: its version field (the
    // first 4 bytes) for a mutable block, and the whole stored block only
    // when it conflicts
    const uint32_t version = view_replica(v, n).version;
    bool stored_newer = false;
    uint32_t stored_version = 0;
    auto head = [&](const uint8_t* p, size_t pn) {
      if (pn < 4) throw ValidationFailed("stored value is no replica");
      std::memcpy(&stored_version, p, 4);
      stored_newer = stored_version >= version;
    };
    if (!storage().read_prefix(k, 4, head) || !k.mutable_block() || !stored_newer) return;
    std::unique_ptr<Block> current;
    auto whole = [&](const uint8_t* p, size_t pn) { current = std::make_unique<Block>(decode_replica(k, p, pn)); };
    if (!storage().read(k, whole)) return;  // erased meanwhile
    throw Conflict("stored version " + std::to_string(stored_version) + " is not older than " +
                       std::to_string(version),
                   std::move(current));
  }
};
}  // namespace

void validate_replica(const Key& k, const uint8_t* v, size_t n) {
  const ReplicaView r = view_replica(v, n);
  if (k.mutable_block()) return;  // a mutable block's own signature checks are outside this path
  // CHB::_validate (CHB.cc:79-99): the content hashes to the address
  Buffer saltowner(r.salt, r.salt + r.salt_len);
  if (r.owner) saltowner.insert(saltowner.end(), r.owner.value.begin(), r.owner.value.end());
  const auto h = sha256(saltowner.data(), saltowner.size(), r.data, r.data_len);
  if (std::memcmp(h.data(), k.value.data(), 31) != 0) throw ValidationFailed("CHB address mismatch");
}

std::string ReplicationConsensus::redundancy() {
  return to_json({{"type", "replication"}, {"desired_factor", std::to_string(factor_)}});
}

std::string ReplicationConsensus::stats() {
  return to_json({{"type", "replication"}, {"factor", std::to_string(factor_)}});
}

std::unique_ptr<Local> ReplicationConsensus::make_local(std::optional<int> port,
                                                        std::optional<IpAddress> listen_address,
                                                        std::unique_ptr<Silo> storage) {
  return std::make_unique<ReplicaLocal>(std::move(storage), port, std::move(listen_address));
}

std::unique_ptr<Local> make_replica_local(std::unique_ptr<Silo> storage) {
  return std::make_unique<ReplicaLocal>(std::move(storage));
}

void ReplicationConsensus::_store(std::unique_ptr<Block> block, StoreMode mode,
                                  std::unique_ptr<ConflictResolver> resolver) {
  std::unique_ptr<Block> resolved;  // the resolver's block, once there is one
  for (;;) {
    const Block& b = resolved ? *resolved : *block;
    auto owners = mode == STORE_INSERT ? overlay_.allocate(b.address, factor_)
                                       : overlay_.lookup(b.address, factor_);
    if (owners.empty()) throw TooFewPeers("no storage peer");
    const Buffer rep = encode_replica(b);
    int reached = 0;
    try {
      for (auto& o : owners) {
        try {
          o->store(replica_key(b.address), rep);
          ++reached;
        } catch (Unavailable&) {
        }
      }
    } catch (Conflict& c) {
      // Consensus::_store (Consensus.cc:59-91): the resolver's block, or
      // the conflict to the caller
      if (!resolver || !c.current) throw;
      Block failed = b;
      auto nb = (*resolver)(failed, *c.current);
      if (!nb) throw;
      resolved = std::move(nb);
      mode = STORE_UPDATE;
      continue;
    }
    if (reached == 0) throw TooFewPeers("no owner reachable");
    return;
  }
}

std::unique_ptr<Block> ReplicationConsensus::_fetch(Address a, std::optional<int> local_version) {
  bool any_up = false;
  for (auto& o : overlay_.lookup(a, factor_)) {
    try {
      std::unique_ptr<Block> b;
      bool bad = false;
      auto take = [&](const uint8_t* r, size_t n) {
        try {
          b = std::make_unique<Block>(decode_replica(a, r, n));
        } catch (ValidationFailed&) {
          bad = true;
        }
      };
      if (!o->try_read(replica_key(a), take)) {
        any_up = true;
        continue;
      }
      if (bad || (!b->is_mutable && !chb_valid(a, b->salt, b->owner, b->data))) continue;
      // no newer than the caller's copy: nothing to return (Paxos::_fetch
      // with a local version)
      if (b->is_mutable && local_version && b->version <= *local_version) return nullptr;
      return b;
    } catch (Unavailable&) {
    }
  }
  if (!any_up) throw TooFewPeers("no replica reachable");
  throw MissingBlock("missing block " + a.hex());
}

void ReplicationConsensus::_remove(Address a, RemoveSignature) {
  int count = 0;
  for (auto& o : overlay_.lookup(a, factor_)) {
    try {
      o->remove(replica_key(a));
      ++count;
    } catch (Unavailable&) {
    } catch (silo::MissingKey&) {
    }
  }
  if (!count) throw MissingBlock("remove: no replica of the block");
}

// ----------------------------------------------------------- configuration
std::string to_json(const ConfigMap& m) {
  std::ostringstream s;
  s << "{";
  bool first = true;
  for (auto& kv : m) {
    if (!first) s << ", ";
    first = false;
    s << "\"" << kv.first << "\": ";
    const bool num = !kv.second.empty() &&
                     kv.second.find_first_not_of("0123456789.-") == std::string::npos;
    if (num) s << kv.second;
    else s << "\"" << kv.second << "\"";
  }
  s << "}";
  return s.str();
}

ConfigMap from_json(const std::string& t) {
  // flat objects only: {"key": "string" | number, ...}
  ConfigMap m;
  size_t i = t.find('{');
  if (i == std::string::npos) throw Error("config: expected an object");
  ++i;
  auto skip = [&] {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\t' || t[i] == ',')) ++i;
  };
  while (true) {
    skip();
    if (i >= t.size()) throw Error("config: unterminated object");
    if (t[i] == '}') break;
    if (t[i] != '"') throw Error("config: expected a key");
    const size_t ke = t.find('"', i + 1);
    const std::string key = t.substr(i + 1, ke - i - 1);
    i = t.find(':', ke);
    if (i == std::string::npos) throw Error("config: expected ':'");
    ++i;
    skip();
    std::string val;
    if (t[i] == '"') {
      const size_t ve = t.find('"', i + 1);
      val = t.substr(i + 1, ve - i - 1);
      i = ve + 1;
    } else {
      const size_t ve = t.find_first_of(",}", i);
      val = t.substr(i, ve - i);
      while (!val.empty() && val.back() == ' ') val.pop_back();
      i = ve;
    }
    m[key] = val;
  }
  return m;
}

namespace {
std::map<std::string, ConsensusFactory>& registry() {
  static std::map<std::string, ConsensusFactory> r;
  return r;
}
struct RegisterReplication {
  RegisterReplication() {
    register_consensus("replication", [](Overlay& ov, const ConfigMap& c) {
      auto it = c.find("replication-factor");
      const int f = it == c.end() ? 3 : std::stoi(it->second);
      return std::unique_ptr<Consensus>(new ReplicationConsensus(ov, f));
    });
  }
} register_replication_;
}  // namespace

void register_consensus(const std::string& type, ConsensusFactory f) { registry()[type] = f; }

std::unique_ptr<Consensus> make_consensus(Overlay& overlay, const std::string& json) {
  const auto c = from_json(json);
  auto it = c.find("type");
  if (it == c.end()) throw Error("config: missing \"type\"");
  auto f = registry().find(it->second);
  if (f == registry().end()) throw Error("config: unknown consensus type " + it->second);
  return f->second(overlay, c);
}

}  // namespace memo_host
