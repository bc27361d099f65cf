// tgsim_bridge.cpp — native packet bridge and UDP front end (include/tgsim.h).
//
// In the reference a plan's datagram crosses its container's data interface: veth -> FIB -> netem
// -> HTB -> docker bridge -> the peer's veth (pkg/runner/local_docker.go:706-721, pkg/sidecar/link.go).
// Here the payload bytes stay on the host, the engine sees one 16-B tgsim_pkt per datagram, and
// every delivery the engine drains is matched back to its payload and queued for the destination:
// twice for a netem duplicate, with one bit flipped for a corrupted copy, never for a dropped one.
//
// Layout: payloads are copied into append-only chunks (one per window of sends, freed when the last
// copy queued from it has been received); each datagram in flight is a record found by
// (src, seq) through a per-source window of record ids (sequence numbers are dense per source);
// deliveries wait in per-destination FIFOs until tgsim_bridge_recv moves them out.
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <stdint.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/tgsim.h"

namespace {

constexpr uint32_t kIpUdpHeader = 28;  // what netem and HTB see on top of the payload
constexpr uint32_t kMaxPayload = 0xFFFFu - kIpUdpHeader;

// netem corrupts one random bit of the packet; the bit is a hash of (src, seq, clone) so a run is
// reproducible (testground_amd/bridge.py restates the same function).
uint32_t flip_bit_index(uint32_t src, uint32_t seq, uint32_t clone, uint32_t len) {
  uint32_t h = (src * 0x9E3779B1u) ^ (seq * 0x85EBCA77u) ^ (clone * 0xC2B2AE3Du);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h % (8u * len);
}

struct Chunk {
  std::vector<uint8_t> bytes;
  uint64_t live = 0;   // datagrams in flight + queued deliveries referencing it
  bool open = true;    // still receiving sends
};

struct Rec {
  uint32_t chunk;
  uint32_t len;
  uint64_t off;
  uint32_t copies;     // deliveries still to come (0: not yet stepped)
  uint32_t src, seq, dst;
};

struct Msg {
  uint64_t t_ns;
  uint32_t src, seq;
  uint16_t flags;
  uint32_t chunk, len;
  uint64_t off;
};

// Growable FIFO ring (power-of-two capacity): the per-source record windows and the
// per-destination inboxes.  Cheaper than std::deque for random access and push/pop.
template <class T>
struct Ring {
  std::vector<T> v;
  uint32_t head = 0, count = 0;
  bool empty() const { return count == 0; }
  uint32_t size() const { return count; }
  T& at(uint32_t k) { return v[(head + k) & (v.size() - 1)]; }
  const T& at(uint32_t k) const { return v[(head + k) & (v.size() - 1)]; }
  T& front() { return v[head]; }
  void pop_front() {
    head = (head + 1) & static_cast<uint32_t>(v.size() - 1);
    --count;
  }
  void push_back(const T& x) {
    if (count == v.size()) grow();
    v[(head + count) & (v.size() - 1)] = x;
    ++count;
  }
  void grow() {
    std::vector<T> n(v.empty() ? 16 : 2 * v.size());
    for (uint32_t k = 0; k < count; ++k) n[k] = at(k);
    v.swap(n);
    head = 0;
  }
};

// Per-source window of record ids, indexed by seq - base (sequence numbers are dense per source).
struct SeqWindow {
  uint32_t base = 0;
  Ring<uint32_t> ids;  // UINT32_MAX: resolved
};

}  // namespace

struct tgsim_bridge_s {
  void* eng = nullptr;
  tgsim_engine_ops ops{};
  uint32_t n = 0, window = 0;
  uint64_t now_tick = 0;
  std::vector<uint32_t> next_seq;
  std::vector<SeqWindow> seqwin;
  std::vector<Rec> recs;
  std::vector<uint32_t> free_recs;
  std::vector<std::unique_ptr<Chunk>> chunks;  // index = chunk id (freed chunks are reset)
  std::vector<uint32_t> free_chunks;
  uint32_t cur_chunk = UINT32_MAX;
  struct Pending {
    tgsim_pkt p;
    uint64_t tick;
    uint32_t rec;
  };
  std::vector<Pending> pending;
  std::vector<Ring<Msg>> inbox;
  uint64_t queued = 0, in_flight = 0;
  std::vector<tgsim_pkt> sub;
  std::vector<uint32_t> sub_rec;
  std::vector<uint8_t> verd;
  std::vector<tgsim_delivery> drained;
};

using Br = tgsim_bridge_s;

namespace {

uint32_t new_chunk(Br* B) {
  uint32_t id;
  if (!B->free_chunks.empty()) {
    id = B->free_chunks.back();
    B->free_chunks.pop_back();
    B->chunks[id]->bytes.clear();
    B->chunks[id]->live = 0;
    B->chunks[id]->open = true;
  } else {
    id = static_cast<uint32_t>(B->chunks.size());
    B->chunks.emplace_back(new Chunk());
  }
  return id;
}

// A freed chunk keeps its memory for the next window's sends (no page faults in steady state).
void chunk_free(Br* B, uint32_t id) {
  B->chunks[id]->bytes.clear();
  B->free_chunks.push_back(id);
}

void chunk_release(Br* B, uint32_t id) {
  Chunk& c = *B->chunks[id];
  if (--c.live == 0 && !c.open) chunk_free(B, id);
}

void resolve(Br* B, uint32_t rid) {
  Rec& r = B->recs[rid];
  SeqWindow& w = B->seqwin[r.src];
  w.ids.at(r.seq - w.base) = UINT32_MAX;
  while (!w.ids.empty() && w.ids.front() == UINT32_MAX) {
    w.ids.pop_front();
    w.base++;
  }
  B->free_recs.push_back(rid);
  B->in_flight--;
}

uint32_t find_rec(const Br* B, uint32_t src, uint32_t seq) {
  if (src >= B->n) return UINT32_MAX;
  const SeqWindow& w = B->seqwin[src];
  const uint32_t k = seq - w.base;
  if (seq < w.base || k >= w.ids.size()) return UINT32_MAX;
  return w.ids.at(k);
}

}  // namespace

extern "C" {

int tgsim_submit(void* engine, const tgsim_pkt* pkts, size_t n);
int tgsim_step(void* engine, uint32_t n_ticks);
int64_t tgsim_verdicts(void* engine, uint8_t* out, size_t cap);
int64_t tgsim_drain(void* engine, tgsim_delivery* out, size_t cap);

int tgsim_bridge_create(void* engine, const tgsim_engine_ops* ops, uint32_t n_peers, uint32_t window_ticks,
                        uint64_t now_tick, void** out) {
  if (!engine || !out || n_peers == 0 || window_ticks == 0 || window_ticks > 0xFFFFu) return -EINVAL;
  Br* B = new Br();
  B->eng = engine;
  if (ops) {
    B->ops = *ops;
  } else {
    B->ops.submit = tgsim_submit;
    B->ops.step = tgsim_step;
    B->ops.verdicts = tgsim_verdicts;
    B->ops.drain = tgsim_drain;
  }
  if (!B->ops.submit || !B->ops.step || !B->ops.verdicts || !B->ops.drain) {
    delete B;
    return -EINVAL;
  }
  B->n = n_peers;
  B->window = window_ticks;
  B->now_tick = now_tick;
  B->next_seq.assign(n_peers, 0);
  B->seqwin.resize(n_peers);
  B->inbox.resize(n_peers);
  *out = B;
  return 0;
}

void tgsim_bridge_destroy(void* b) { delete static_cast<Br*>(b); }

int64_t tgsim_bridge_send(void* b, size_t n, const uint32_t* src, const uint32_t* dst, const uint8_t* data,
                          const uint64_t* off, const uint64_t* ticks, uint32_t* seq_out) {
  Br* B = static_cast<Br*>(b);
  if (!B || (n && (!src || !dst || !off || (!data && off[n] > off[0])))) return -EINVAL;
  for (size_t i = 0; i < n; ++i) {  // validate the whole batch first: all or nothing
    if (src[i] >= B->n || (dst[i] != TGSIM_EXTERNAL && dst[i] >= B->n)) return -EINVAL;
    if (off[i + 1] < off[i] || off[i + 1] - off[i] > kMaxPayload) return -EMSGSIZE;
    if (ticks && ticks[i] < B->now_tick) return -EINVAL;
    if (B->next_seq[src[i]] == UINT32_MAX) return -EOVERFLOW;
  }
  if (B->cur_chunk == UINT32_MAX) B->cur_chunk = new_chunk(B);
  Chunk& c = *B->chunks[B->cur_chunk];
  const uint64_t base = c.bytes.size();
  c.bytes.insert(c.bytes.end(), data + off[0], data + off[n]);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t s = src[i], len = static_cast<uint32_t>(off[i + 1] - off[i]);
    const uint32_t seq = B->next_seq[s]++;
    uint32_t rid;
    if (!B->free_recs.empty()) {
      rid = B->free_recs.back();
      B->free_recs.pop_back();
    } else {
      rid = static_cast<uint32_t>(B->recs.size());
      B->recs.emplace_back();
    }
    B->recs[rid] = Rec{B->cur_chunk, len, base + (off[i] - off[0]), 0, s, seq, dst[i]};
    SeqWindow& w = B->seqwin[s];
    if (w.ids.empty()) w.base = seq;
    w.ids.push_back(rid);
    c.live++;
    B->in_flight++;
    tgsim_pkt p;
    p.src = s;
    p.dst = dst[i];
    p.seq = seq;
    p.len = static_cast<uint16_t>(len + kIpUdpHeader);
    p.tick = 0;
    B->pending.push_back({p, ticks ? ticks[i] : B->now_tick, rid});
    if (seq_out) seq_out[i] = seq;
  }
  return static_cast<int64_t>(n);
}

int64_t tgsim_bridge_step(void* b) {
  Br* B = static_cast<Br*>(b);
  if (!B) return -EINVAL;
  const uint64_t end = B->now_tick + B->window;
  B->sub.clear();
  B->sub_rec.clear();
  size_t keep = 0;
  for (size_t i = 0; i < B->pending.size(); ++i) {
    Br::Pending& q = B->pending[i];
    if (q.tick < end) {
      q.p.tick = static_cast<uint16_t>(q.tick - B->now_tick);
      B->sub.push_back(q.p);
      B->sub_rec.push_back(q.rec);
    } else {
      B->pending[keep++] = q;
    }
  }
  B->pending.resize(keep);
  if (B->cur_chunk != UINT32_MAX) {  // this window's sends are complete: the chunk closes
    Chunk& c = *B->chunks[B->cur_chunk];
    c.open = false;
    if (c.live == 0) chunk_free(B, B->cur_chunk);
    B->cur_chunk = UINT32_MAX;
  }
  int rc = 0;
  if (!B->sub.empty() && (rc = B->ops.submit(B->eng, B->sub.data(), B->sub.size()))) return rc;
  if ((rc = B->ops.step(B->eng, B->window))) return rc;
  B->now_tick = end;
  if (!B->sub.empty()) {
    B->verd.resize(B->sub.size());
    const int64_t nv = B->ops.verdicts(B->eng, B->verd.data(), B->verd.size());
    if (nv < 0) return nv;
    if (static_cast<size_t>(nv) != B->sub.size()) return -EIO;
    for (size_t i = 0; i < B->sub.size(); ++i) {
      const uint8_t v = B->verd[i];
      const uint32_t copies = ((v & 15u) == TGSIM_V_SCHEDULED ? 1u : 0u) + ((v >> 4) == TGSIM_V_SCHEDULED ? 1u : 0u);
      const uint32_t rid = B->sub_rec[i];
      if (copies) {
        B->recs[rid].copies = copies;
      } else {  // dropped, filtered or queue-full: no copy will ever arrive
        const uint32_t ch = B->recs[rid].chunk;
        resolve(B, rid);
        chunk_release(B, ch);
      }
    }
  }
  int64_t total = 0;
  if (B->drained.size() < 65536) B->drained.resize(65536);
  for (;;) {
    const int64_t k = B->ops.drain(B->eng, B->drained.data(), B->drained.size());
    if (k < 0) return k;
    for (int64_t i = 0; i < k; ++i) {
      const tgsim_delivery& d = B->drained[i];
      const uint32_t rid = find_rec(B, d.src, d.seq);
      if (rid == UINT32_MAX || d.dst >= B->n) return -EIO;  // a delivery the bridge never sent
      Rec& r = B->recs[rid];
      B->inbox[d.dst].push_back(Msg{d.t_ns, d.src, d.seq, d.flags, r.chunk, r.len, r.off});
      B->chunks[r.chunk]->live++;  // the queued message holds the payload
      B->queued++;
      if (--r.copies == 0) {
        const uint32_t ch = r.chunk;
        resolve(B, rid);
        chunk_release(B, ch);
      }
    }
    total += k;
    if (static_cast<size_t>(k) < B->drained.size()) break;
  }
  return total;
}

int64_t tgsim_bridge_recv(void* b, uint32_t peer, tgsim_msg* msgs, size_t max, uint8_t* data, size_t cap) {
  Br* B = static_cast<Br*>(b);
  if (!B || (max && !msgs) || (cap && !data) || (peer != UINT32_MAX && peer >= B->n)) return -EINVAL;
  size_t k = 0, used = 0;
  const uint32_t p0 = peer == UINT32_MAX ? 0 : peer, p1 = peer == UINT32_MAX ? B->n : peer + 1;
  for (uint32_t p = p0; p < p1 && k < max; ++p) {
    Ring<Msg>& q = B->inbox[p];
    while (!q.empty() && k < max) {
      const Msg& m = q.front();
      if (used + m.len > cap) return static_cast<int64_t>(k);  // the caller's buffer is full
      memcpy(data + used, B->chunks[m.chunk]->bytes.data() + m.off, m.len);
      if ((m.flags & TGSIM_FLAG_CORRUPT) && m.len) {
        const uint32_t bit = flip_bit_index(m.src, m.seq, m.flags & TGSIM_FLAG_DUP, m.len);
        data[used + (bit >> 3)] ^= static_cast<uint8_t>(1u << (bit & 7));
      }
      tgsim_msg& o = msgs[k++];
      o.t_ns = m.t_ns;
      o.src = m.src;
      o.dst = p;
      o.seq = m.seq;
      o.flags = m.flags;
      o._pad = 0;
      o.off = used;
      o.len = m.len;
      o._pad2 = 0;
      used += m.len;
      chunk_release(B, m.chunk);
      q.pop_front();
      B->queued--;
    }
  }
  return static_cast<int64_t>(k);
}

int64_t tgsim_bridge_pending(void* b, uint32_t peer) {
  Br* B = static_cast<Br*>(b);
  if (!B || (peer != UINT32_MAX && peer >= B->n)) return -EINVAL;
  return peer == UINT32_MAX ? static_cast<int64_t>(B->queued) : static_cast<int64_t>(B->inbox[peer].size());
}

int64_t tgsim_bridge_in_flight(void* b) {
  Br* B = static_cast<Br*>(b);
  return B ? static_cast<int64_t>(B->in_flight) : -EINVAL;
}

int64_t tgsim_bridge_link_removed(void* b, uint32_t peer) {
  Br* B = static_cast<Br*>(b);
  if (!B || peer >= B->n) return -EINVAL;
  // records awaiting a delivery (copies > 0) were handed to the engine and given a SCHEDULED
  // verdict; the engine's flush (sender side) and purge (destination side) drop them silently
  int64_t k = 0;
  for (uint32_t rid = 0; rid < B->recs.size(); ++rid) {
    Rec& r = B->recs[rid];
    if (r.copies == 0 || (r.src != peer && r.dst != peer)) continue;
    r.copies = 0;
    const uint32_t ch = r.chunk;
    resolve(B, rid);
    chunk_release(B, ch);
    ++k;
  }
  return k;
}

uint64_t tgsim_bridge_now_tick(void* b) {
  Br* B = static_cast<Br*>(b);
  return B ? B->now_tick : 0;
}

// ---- UDP front end ---------------------------------------------------------------------------
struct tgsim_udp_front_s {
  Br* br = nullptr;
  int fd = -1;
  uint16_t port = 0;
  std::vector<sockaddr_in> addr;                // per peer (sin_port 0: unregistered)
  std::unordered_map<uint64_t, uint32_t> peer;  // (ip << 16 | port) -> peer
  // batches
  static constexpr unsigned kBatch = 512;
  std::vector<uint8_t> rxbuf;
  std::vector<mmsghdr> rxh;
  std::vector<iovec> rxv;
  std::vector<sockaddr_in> rxa;
  std::vector<uint32_t> s_src, s_dst;
  std::vector<uint64_t> s_off;
  std::vector<uint8_t> s_data;
  std::vector<tgsim_msg> msgs;
  std::vector<uint8_t> payload;
  std::vector<uint32_t> hdr;
  std::vector<mmsghdr> txh;
  std::vector<iovec> txv;
  // header-less mode: peer p's data address is a socket of the front end (vfd[p]); what arrives
  // there is addressed to p, and what is delivered from p leaves from it
  std::vector<int> vfd;                          // per peer, -1: none
  std::unordered_map<int, uint32_t> vpeer;       // fd -> peer
  int ep = -1;                                   // epoll set of the vfd sockets
};
using Uf = tgsim_udp_front_s;

int tgsim_udp_front_create(void* bridge, uint16_t port, void** out) {
  if (!bridge || !out) return -EINVAL;
  Uf* F = new Uf();
  F->br = static_cast<Br*>(bridge);
  F->fd = socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK, 0);
  if (F->fd < 0) {
    const int e = errno;
    delete F;
    return -e;
  }
  int sz = 16 << 20;
  (void)setsockopt(F->fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
  (void)setsockopt(F->fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = htons(port);
  socklen_t al = sizeof a;
  if (bind(F->fd, reinterpret_cast<sockaddr*>(&a), sizeof a) || getsockname(F->fd, reinterpret_cast<sockaddr*>(&a), &al)) {
    const int e = errno;
    close(F->fd);
    delete F;
    return -e;
  }
  F->port = ntohs(a.sin_port);
  F->addr.assign(F->br->n, sockaddr_in{});
  F->vfd.assign(F->br->n, -1);
  F->rxbuf.resize(static_cast<size_t>(Uf::kBatch) * 65536);
  F->rxh.resize(Uf::kBatch);
  F->rxv.resize(Uf::kBatch);
  F->rxa.resize(Uf::kBatch);
  *out = F;
  return 0;
}

int tgsim_udp_front_port(void* f) { return f ? static_cast<Uf*>(f)->port : -EINVAL; }

int tgsim_udp_front_register(void* f, uint32_t peer, uint32_t ipv4, uint16_t port) {
  Uf* F = static_cast<Uf*>(f);
  if (!F || peer >= F->br->n || !port) return -EINVAL;
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(ipv4);
  a.sin_port = htons(port);
  F->addr[peer] = a;
  F->peer[(static_cast<uint64_t>(ipv4) << 16) | port] = peer;
  return 0;
}

int tgsim_udp_front_bind_peer(void* f, uint32_t peer, uint32_t ipv4, uint16_t port) {
  Uf* F = static_cast<Uf*>(f);
  if (!F || peer >= F->br->n || F->vfd[peer] >= 0) return -EINVAL;
  if (F->ep < 0 && (F->ep = epoll_create1(0)) < 0) return -errno;
  const int fd = socket(AF_INET, SOCK_DGRAM | SOCK_NONBLOCK, 0);
  if (fd < 0) return -errno;
  int sz = 4 << 20;
  (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(ipv4);
  a.sin_port = htons(port);
  socklen_t al = sizeof a;
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = fd;
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) || getsockname(fd, reinterpret_cast<sockaddr*>(&a), &al) ||
      epoll_ctl(F->ep, EPOLL_CTL_ADD, fd, &ev)) {
    const int e = errno;
    close(fd);
    return -e;
  }
  F->vfd[peer] = fd;
  F->vpeer[fd] = peer;
  return ntohs(a.sin_port);
}

namespace {
// The datagrams waiting on one socket, in recvmmsg batches, into bridge sends.  dst_fixed:
// UINT32_MAX for the header socket (a 4-byte destination header leads each datagram), else the peer
// whose data-address socket this is (the payload is the whole datagram).
int64_t drain_socket(Uf* F, int fd, uint32_t dst_fixed) {
  for (;;) {
    for (unsigned i = 0; i < Uf::kBatch; ++i) {
      F->rxv[i].iov_base = F->rxbuf.data() + static_cast<size_t>(i) * 65536;
      F->rxv[i].iov_len = 65536;
      memset(&F->rxh[i], 0, sizeof(mmsghdr));
      F->rxh[i].msg_hdr.msg_iov = &F->rxv[i];
      F->rxh[i].msg_hdr.msg_iovlen = 1;
      F->rxh[i].msg_hdr.msg_name = &F->rxa[i];
      F->rxh[i].msg_hdr.msg_namelen = sizeof(sockaddr_in);
    }
    const int got = recvmmsg(fd, F->rxh.data(), Uf::kBatch, MSG_DONTWAIT, nullptr);
    if (got <= 0) break;
    F->s_src.clear();
    F->s_dst.clear();
    F->s_data.clear();
    F->s_off.assign(1, 0);
    const size_t hdr = dst_fixed == UINT32_MAX ? 4 : 0;
    for (int i = 0; i < got; ++i) {
      const size_t len = F->rxh[i].msg_len;
      const sockaddr_in& sa = F->rxa[i];
      auto it = F->peer.find((static_cast<uint64_t>(ntohl(sa.sin_addr.s_addr)) << 16) | ntohs(sa.sin_port));
      if (it == F->peer.end() || len < hdr) continue;  // not an instance of this run
      const uint8_t* m = F->rxbuf.data() + static_cast<size_t>(i) * 65536;
      uint32_t dst = dst_fixed;
      if (hdr) {
        memcpy(&dst, m, 4);
        dst = ntohl(dst);
      }
      if (dst != TGSIM_EXTERNAL && dst >= F->br->n) continue;
      if (len - hdr > kMaxPayload) continue;
      F->s_src.push_back(it->second);
      F->s_dst.push_back(dst);
      F->s_data.insert(F->s_data.end(), m + hdr, m + len);
      F->s_off.push_back(F->s_data.size());
    }
    if (!F->s_src.empty()) {
      const int64_t rc = tgsim_bridge_send(F->br, F->s_src.size(), F->s_src.data(), F->s_dst.data(), F->s_data.data(),
                                           F->s_off.data(), nullptr, nullptr);
      if (rc < 0) return rc;
    }
    if (got < static_cast<int>(Uf::kBatch)) break;
  }
  return 0;
}

// sendmmsg of txh[i0, i1) from fd, waiting for room when the socket buffer is full.
int send_all(int fd, mmsghdr* h, size_t m) {
  for (size_t i = 0; i < m;) {
    const int sent = sendmmsg(fd, h + i, static_cast<unsigned>(std::min<size_t>(m - i, 1024)), 0);
    if (sent < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == ENOBUFS) {
        pollfd pf{fd, POLLOUT, 0};
        if (poll(&pf, 1, 1000) <= 0) return -EAGAIN;
        continue;
      }
      return -errno;
    }
    i += static_cast<size_t>(sent);
  }
  return 0;
}
}  // namespace

int64_t tgsim_udp_front_pump(void* f) {
  Uf* F = static_cast<Uf*>(f);
  if (!F) return -EINVAL;
  // ---- everything that arrived: the header socket, then every ready data-address socket
  int64_t rc = drain_socket(F, F->fd, UINT32_MAX);
  if (rc < 0) return rc;
  if (F->ep >= 0) {
    epoll_event evs[256];
    for (;;) {
      const int k = epoll_wait(F->ep, evs, 256, 0);
      if (k < 0 && errno == EINTR) continue;
      if (k <= 0) break;
      for (int i = 0; i < k; ++i)
        if ((rc = drain_socket(F, evs[i].data.fd, F->vpeer[evs[i].data.fd])) < 0) return rc;
      if (k < 256) break;
    }
  }
  const int64_t n = tgsim_bridge_step(F->br);
  if (n < 0) return n;
  // ---- deliveries to the registered addresses, sendmmsg batches (4-byte source header + payload)
  const size_t q = F->br->queued;
  if (!q) return n;
  F->msgs.resize(q);
  size_t bytes = 0;
  for (uint32_t p = 0; p < F->br->n; ++p)
    for (uint32_t k = 0; k < F->br->inbox[p].size(); ++k) bytes += F->br->inbox[p].at(k).len;
  F->payload.resize(bytes ? bytes : 1);
  const int64_t k = tgsim_bridge_recv(F->br, UINT32_MAX, F->msgs.data(), q, F->payload.data(), F->payload.size());
  if (k < 0) return k;
  F->hdr.resize(static_cast<size_t>(k));
  F->txh.resize(static_cast<size_t>(k));
  F->txv.resize(2 * static_cast<size_t>(k));
  // deliveries from a source with a data-address socket leave from it, without a header (the
  // receiver's recvfrom sees the source's address); the others leave from the header socket.  They
  // go out in delivery order (each destination's datagrams in simulated-time order, across senders
  // too): a sendmmsg batch is flushed whenever the sending socket changes.
  size_t m = 0;
  int cur = -2;
  size_t run0 = 0;
  for (int64_t r = 0; r <= k; ++r) {
    const int fd = r < k ? F->vfd[F->msgs[r].src] : -3;
    if (fd != cur) {  // flush the run of the previous socket
      if (m > run0) {
        const int rc2 = send_all(cur < 0 ? F->fd : cur, F->txh.data() + run0, m - run0);
        if (rc2) return rc2;
      }
      run0 = m;
      cur = fd;
    }
    if (r == k) break;
    const tgsim_msg& g = F->msgs[r];
    sockaddr_in& to = F->addr[g.dst];
    if (!to.sin_port) continue;  // nobody listening for that instance
    memset(&F->txh[m], 0, sizeof(mmsghdr));
    if (fd < 0) {
      F->hdr[m] = htonl(g.src);
      F->txv[2 * m] = iovec{&F->hdr[m], 4};
      F->txv[2 * m + 1] = iovec{F->payload.data() + g.off, g.len};
      F->txh[m].msg_hdr.msg_iov = &F->txv[2 * m];
      F->txh[m].msg_hdr.msg_iovlen = 2;
    } else {
      F->txv[2 * m] = iovec{F->payload.data() + g.off, g.len};
      F->txh[m].msg_hdr.msg_iov = &F->txv[2 * m];
      F->txh[m].msg_hdr.msg_iovlen = 1;
    }
    F->txh[m].msg_hdr.msg_name = &to;
    F->txh[m].msg_hdr.msg_namelen = sizeof to;
    ++m;
  }
  return n;
}

void tgsim_udp_front_destroy(void* f) {
  Uf* F = static_cast<Uf*>(f);
  if (!F) return;
  if (F->fd >= 0) close(F->fd);
  for (int fd : F->vfd)
    if (fd >= 0) close(fd);
  if (F->ep >= 0) close(F->ep);
  delete F;
}

}  // extern "C"
