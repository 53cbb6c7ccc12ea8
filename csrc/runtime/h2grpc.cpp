#include "h2grpc.h"
#include "thread_name.h"

#include <arpa/inet.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <unordered_map>

namespace igp {

// ---------------------------------------------------------------------------- libnghttp2 (dlopen)
// The ABI-stable subset of nghttp2.h this server uses (libnghttp2.so.14).
namespace {

struct NgFrameHd {
  size_t length;
  int32_t stream_id;
  uint8_t type;
  uint8_t flags;
  uint8_t reserved;
};
struct NgNv {
  const uint8_t* name;
  const uint8_t* value;
  size_t namelen;
  size_t valuelen;
  uint8_t flags;
};
union NgDataSource {
  int fd;
  void* ptr;
};
typedef ssize_t (*NgReadCb)(void* session, int32_t stream_id, uint8_t* buf, size_t length, uint32_t* data_flags,
                            NgDataSource* source, void* user_data);
struct NgDataProvider {
  NgDataSource source;
  NgReadCb read_callback;
};
struct NgSettingsEntry {
  int32_t settings_id;
  uint32_t value;
};
constexpr uint8_t kFrameData = 0, kFrameHeaders = 1, kFlagEndStream = 0x01;
constexpr uint32_t kDataEof = 0x01, kDataNoEndStream = 0x02;
constexpr int32_t kSettingsMaxStreams = 0x03, kSettingsInitialWindow = 0x04;

struct Ng {
  int (*callbacks_new)(void**);
  void (*callbacks_del)(void*);
  void (*set_on_begin_headers)(void*, int (*)(void*, const void*, void*));
  void (*set_on_header)(void*, int (*)(void*, const void*, const uint8_t*, size_t, const uint8_t*, size_t, uint8_t, void*));
  void (*set_on_data_chunk_recv)(void*, int (*)(void*, uint8_t, int32_t, const uint8_t*, size_t, void*));
  void (*set_on_frame_recv)(void*, int (*)(void*, const void*, void*));
  void (*set_on_stream_close)(void*, int (*)(void*, int32_t, uint32_t, void*));
  int (*server_new)(void**, const void*, void*);
  int (*client_new)(void**, const void*, void*);
  int32_t (*submit_request)(void*, const void*, const NgNv*, size_t, const NgDataProvider*, void*);
  void* (*stream_user_data)(void*, int32_t);
  void (*session_del)(void*);
  ssize_t (*mem_recv)(void*, const uint8_t*, size_t);
  ssize_t (*mem_send)(void*, const uint8_t**);
  int (*submit_settings)(void*, uint8_t, const NgSettingsEntry*, size_t);
  int (*submit_response)(void*, int32_t, const NgNv*, size_t, const NgDataProvider*);
  int (*submit_trailer)(void*, int32_t, const NgNv*, size_t);
  int (*want_read)(void*);
  int (*want_write)(void*);
  int (*set_local_window_size)(void*, uint8_t, int32_t, int32_t);  // optional (nghttp2 >= 1.11)
};

const Ng& ng() {
  static Ng n{};
  static bool loaded = false;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (loaded) return n;
  void* h = dlopen("libnghttp2.so.14", RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error(std::string("grpc server: cannot load libnghttp2: ") + dlerror());
  auto sym = [&](const char* name) {
    void* f = dlsym(h, name);
    if (!f) throw std::runtime_error(std::string("grpc server: libnghttp2 lacks ") + name);
    return f;
  };
#define NG_SYM(field, name) n.field = reinterpret_cast<decltype(n.field)>(sym(name))
  NG_SYM(callbacks_new, "nghttp2_session_callbacks_new");
  NG_SYM(callbacks_del, "nghttp2_session_callbacks_del");
  NG_SYM(set_on_begin_headers, "nghttp2_session_callbacks_set_on_begin_headers_callback");
  NG_SYM(set_on_header, "nghttp2_session_callbacks_set_on_header_callback");
  NG_SYM(set_on_data_chunk_recv, "nghttp2_session_callbacks_set_on_data_chunk_recv_callback");
  NG_SYM(set_on_frame_recv, "nghttp2_session_callbacks_set_on_frame_recv_callback");
  NG_SYM(set_on_stream_close, "nghttp2_session_callbacks_set_on_stream_close_callback");
  NG_SYM(server_new, "nghttp2_session_server_new");
  NG_SYM(client_new, "nghttp2_session_client_new");
  NG_SYM(submit_request, "nghttp2_submit_request");
  NG_SYM(stream_user_data, "nghttp2_session_get_stream_user_data");
  NG_SYM(session_del, "nghttp2_session_del");
  NG_SYM(mem_recv, "nghttp2_session_mem_recv");
  NG_SYM(mem_send, "nghttp2_session_mem_send");
  NG_SYM(submit_settings, "nghttp2_submit_settings");
  NG_SYM(submit_response, "nghttp2_submit_response");
  NG_SYM(submit_trailer, "nghttp2_submit_trailer");
  NG_SYM(want_read, "nghttp2_session_want_read");
  NG_SYM(want_write, "nghttp2_session_want_write");
#undef NG_SYM
  n.set_local_window_size = reinterpret_cast<decltype(n.set_local_window_size)>(dlsym(h, "nghttp2_session_set_local_window_size"));
  loaded = true;
  return n;
}

NgNv nv(const char* name, const std::string& value) {
  return NgNv{reinterpret_cast<const uint8_t*>(name), reinterpret_cast<const uint8_t*>(value.data()), std::strlen(name),
              value.size(), 0};
}

// grpc-message is percent-encoded (printable ASCII except '%' passes through)
std::string pct(const std::string& s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  for (unsigned char c : s) {
    if (c >= 0x20 && c <= 0x7e && c != '%') {
      o += char(c);
    } else {
      o += '%';
      o += hex[c >> 4];
      o += hex[c & 15];
    }
  }
  return o;
}

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

constexpr uint64_t kTagListen = 1, kTagEvent = 2, kFirstConn = 16;
constexpr int kWorkerShift = 40;
constexpr uint64_t kTokenMask = (uint64_t(1) << kWorkerShift) - 1;
const std::string kPathTx = "/risk.v1.RiskService/ScoreTransaction";
const std::string kPathBatch = "/risk.v1.RiskService/ScoreBatch";
const std::string kPathLtv = "/risk.v1.RiskService/PredictLTV";
const std::string kPathSeg = "/risk.v1.RiskService/GetPlayerSegment";
const std::string kPathAbuse = "/risk.v1.RiskService/CheckBonusAbuse";

// the account RPC a path names (0: none)
uint8_t acct_rpc(const std::string& path) {
  if (path == kPathLtv) return RPC_LTV;
  if (path == kPathSeg) return RPC_SEGMENT;
  if (path == kPathAbuse) return RPC_ABUSE;
  return 0;
}

// a failed hot call: malformed requests answer INVALID_ARGUMENT; anything else (a device error or
// deadline inside a core) is retried through the cold handler table
bool invalid_request(const std::string& err) {
  return err.rfind("invalid: ", 0) == 0 || err.find("pb:") != std::string::npos;
}
std::string invalid_message(const std::string& err) {
  return err.rfind("invalid: ", 0) == 0 ? err.substr(9) : err;
}

}  // namespace

// ---------------------------------------------------------------------------- worker
struct GrpcServer::Worker {
  struct Stream {
    std::string path;
    std::string data;
    std::string out;  // 5-byte prefix + response message
    size_t off = 0;
  };
  struct Conn {
    Worker* w = nullptr;
    uint64_t id = 0;
    int fd = -1;
    void* sess = nullptr;
    std::unordered_map<int32_t, Stream> streams;
    std::string wbuf;
    size_t woff = 0;
    bool epollout = false;
    size_t buffered = 0;  // request bytes held by this connection's streams
  };
  struct Done {
    uint64_t token;  // hot unary: pending-table token; 0: conn / stream below
    uint64_t conn;
    int32_t stream;
    GrpcReply reply;
    bool retry = false;  // a failed hot call: run it again through the cold handler table
    bool cold = false;   // ... because no native core can serve it (no failover: kColdPrefix)
  };
  struct Pend {  // a hot unary call in a core: where to answer, and its request for a retry
    uint64_t conn;
    int32_t stream;
    std::string path;
    std::string body;
  };

  GrpcServer* srv;
  int idx;
  int lfd = -1, ep = -1, evfd = -1;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
  uint64_t next_conn = kFirstConn;
  std::unordered_map<uint64_t, Pend> pending;  // token -> the call
  uint64_t next_token = 1;
  std::mutex qmu;
  std::vector<Done> q;
  std::atomic<bool> stop{false};
  void* cbs = nullptr;

  Worker(GrpcServer* s, int i) : srv(s), idx(i) {}
  ~Worker() {
    for (auto& kv : conns) close_conn_raw(*kv.second);
    conns.clear();
    if (cbs) ng().callbacks_del(cbs);
    if (lfd >= 0) ::close(lfd);
    if (ep >= 0) ::close(ep);
    if (evfd >= 0) ::close(evfd);
  }

  // unary ScoreTransaction calls completed by one read() (dispatch), handed to the core at once
  std::vector<ServeCore::TxCall> txq;
  void submit_txq() {
    if (txq.empty()) return;
    srv->core_->submit_tx_many(txq.data(), txq.size(), -1);
    txq.clear();
  }

  // completions from other threads; the eventfd is written only when the queue was empty (a
  // non-empty queue already has a wake-up pending and drain_done takes all of it): one syscall
  // per burst of completions instead of one per call
  void post(Done&& d) {
    bool wake;
    {
      std::lock_guard<std::mutex> g(qmu);
      wake = q.empty();
      q.push_back(std::move(d));
    }
    if (wake) notify();
  }
  void post_many(std::vector<Done>& ds) {
    if (ds.empty()) return;
    bool wake;
    {
      std::lock_guard<std::mutex> g(qmu);
      wake = q.empty();
      for (auto& d : ds) q.push_back(std::move(d));
    }
    ds.clear();
    if (wake) notify();
  }
  void notify() {
    const uint64_t one = 1;
    ssize_t r = ::write(evfd, &one, sizeof one);
    (void)r;
  }

  // ---- nghttp2 callbacks (user_data = Conn*)
  static int on_begin_headers(void*, const void* frame, void* ud) {
    auto* c = static_cast<Conn*>(ud);
    const auto* hd = static_cast<const NgFrameHd*>(frame);
    if (hd->type == kFrameHeaders) c->streams[hd->stream_id];
    return 0;
  }
  static int on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                       size_t valuelen, uint8_t, void* ud) {
    auto* c = static_cast<Conn*>(ud);
    const auto* hd = static_cast<const NgFrameHd*>(frame);
    if (hd->type != kFrameHeaders) return 0;
    if (namelen == 5 && std::memcmp(name, ":path", 5) == 0) {
      auto it = c->streams.find(hd->stream_id);
      if (it != c->streams.end()) it->second.path.assign(reinterpret_cast<const char*>(value), valuelen);
    }
    return 0;
  }
  static int on_data(void*, uint8_t, int32_t sid, const uint8_t* data, size_t len, void* ud) {
    auto* c = static_cast<Conn*>(ud);
    auto it = c->streams.find(sid);
    if (it != c->streams.end()) {
      // per-stream (64 MiB) and per-connection (kMaxConnBuffered) request bytes: past either the
      // connection fails (NGHTTP2_ERR_CALLBACK_FAILURE) instead of the server allocating without
      // bound
      if (it->second.data.size() + len > (size_t(64) << 20) || c->buffered + len > kMaxConnBuffered) return -902;
      it->second.data.append(reinterpret_cast<const char*>(data), len);
      c->buffered += len;
    }
    return 0;
  }
  static int on_frame(void*, const void* frame, void* ud) {
    auto* c = static_cast<Conn*>(ud);
    const auto* hd = static_cast<const NgFrameHd*>(frame);
    if ((hd->type == kFrameData || hd->type == kFrameHeaders) && (hd->flags & kFlagEndStream))
      c->w->dispatch(*c, hd->stream_id);
    return 0;
  }
  static int on_close(void*, int32_t sid, uint32_t, void* ud) {
    auto* c = static_cast<Conn*>(ud);
    auto it = c->streams.find(sid);
    if (it != c->streams.end()) {
      c->buffered -= std::min(c->buffered, it->second.data.size());
      c->streams.erase(it);
    }
    return 0;
  }
  static ssize_t read_body(void* sess, int32_t sid, uint8_t* buf, size_t len, uint32_t* flags, NgDataSource* src,
                           void*) {
    auto* st = static_cast<Stream*>(src->ptr);
    const size_t n = std::min(len, st->out.size() - st->off);
    std::memcpy(buf, st->out.data() + st->off, n);
    st->off += n;
    if (st->off == st->out.size()) {
      *flags |= kDataEof | kDataNoEndStream;
      static const std::string ok = "0";
      const NgNv tr[1] = {nv("grpc-status", ok)};
      ng().submit_trailer(sess, sid, tr, 1);
    }
    return ssize_t(n);
  }

  void init(const std::string& host, int port) {
    const Ng& n = ng();
    if (n.callbacks_new(&cbs) != 0) throw std::runtime_error("grpc server: nghttp2 callbacks");
    n.set_on_begin_headers(cbs, on_begin_headers);
    n.set_on_header(cbs, on_header);
    n.set_on_data_chunk_recv(cbs, on_data);
    n.set_on_frame_recv(cbs, on_frame);
    n.set_on_stream_close(cbs, on_close);
    lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (lfd < 0) throw std::runtime_error("grpc server: socket");
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(uint16_t(port));
    if (host.empty() || host == "0.0.0.0" || host == "[::]") a.sin_addr.s_addr = htonl(INADDR_ANY);
    else if (::inet_pton(AF_INET, host == "localhost" ? "127.0.0.1" : host.c_str(), &a.sin_addr) != 1)
      throw std::runtime_error("grpc server: bad host " + host);
    if (::bind(lfd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0)
      throw std::runtime_error(std::string("grpc server: bind: ") + std::strerror(errno));
    if (::listen(lfd, 1024) != 0) throw std::runtime_error("grpc server: listen");
    ep = ::epoll_create1(EPOLL_CLOEXEC);
    evfd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (ep < 0 || evfd < 0) throw std::runtime_error("grpc server: epoll / eventfd");
    epoll_event e{};
    e.events = EPOLLIN;
    e.data.u64 = kTagListen;
    ::epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &e);
    e.data.u64 = kTagEvent;
    ::epoll_ctl(ep, EPOLL_CTL_ADD, evfd, &e);
  }
  int bound_port() const {
    sockaddr_in a{};
    socklen_t l = sizeof a;
    ::getsockname(lfd, reinterpret_cast<sockaddr*>(&a), &l);
    return ntohs(a.sin_port);
  }

  void run() {
    epoll_event evs[64];
    std::vector<char> rbuf(size_t(256) << 10);
    while (!stop.load(std::memory_order_relaxed)) {
      const int n = ::epoll_wait(ep, evs, 64, 100);
      for (int i = 0; i < n; ++i) {
        const uint64_t tag = evs[i].data.u64;
        if (tag == kTagListen) {
          accept_all();
        } else if (tag == kTagEvent) {
          uint64_t v;
          ssize_t r = ::read(evfd, &v, sizeof v);
          (void)r;
          drain_done();
        } else {
          auto it = conns.find(tag);
          if (it == conns.end()) continue;
          Conn& c = *it->second;
          bool ok = true;
          if (evs[i].events & EPOLLIN) ok = read_conn(c, rbuf);
          if (ok && (evs[i].events & (EPOLLERR | EPOLLHUP)) && !(evs[i].events & EPOLLIN)) ok = false;
          if (ok) ok = flush(c);
          if (!ok) close_conn(tag);
        }
      }
      submit_txq();  // (calls dispatched outside a read, if any)
    }
  }

  void accept_all() {
    for (;;) {
      const int fd = ::accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->w = this;
      c->id = next_conn++;
      c->fd = fd;
      const Ng& n = ng();
      if (n.server_new(&c->sess, cbs, c.get()) != 0) {
        ::close(fd);
        continue;
      }
      const NgSettingsEntry iv[2] = {{kSettingsMaxStreams, kMaxStreams}, {kSettingsInitialWindow, 8u << 20}};
      n.submit_settings(c->sess, 0, iv, 2);
      if (n.set_local_window_size) n.set_local_window_size(c->sess, 0, 0, 64 << 20);
      epoll_event e{};
      e.events = EPOLLIN;
      e.data.u64 = c->id;
      ::epoll_ctl(ep, EPOLL_CTL_ADD, fd, &e);
      srv->conns_.fetch_add(1, std::memory_order_relaxed);
      Conn& ref = *c;
      conns.emplace(c->id, std::move(c));
      if (!flush(ref)) close_conn(ref.id);
    }
  }

  bool read_conn(Conn& c, std::vector<char>& buf) {
    for (;;) {
      const ssize_t r = ::read(c.fd, buf.data(), buf.size());
      if (r == 0) return false;
      if (r < 0) return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
      const ssize_t k = ng().mem_recv(c.sess, reinterpret_cast<const uint8_t*>(buf.data()), size_t(r));
      submit_txq();  // the unary calls this chunk completed, as one batch
      if (k < 0) return false;
      // a short read drained the socket: no second read() just to see EAGAIN (level-triggered
      // epoll reports the connection again when more bytes arrive)
      if (size_t(r) < buf.size()) return true;
    }
  }

  // write what nghttp2 has queued; the remainder waits for EPOLLOUT
  bool flush(Conn& c) {
    const Ng& n = ng();
    auto write_some = [&](const char* p, size_t len) -> size_t {
      size_t done = 0;
      while (done < len) {
        const ssize_t w = ::send(c.fd, p + done, len - done, MSG_NOSIGNAL);
        if (w < 0) {
          if (errno == EINTR) continue;
          if (errno == EAGAIN || errno == EWOULDBLOCK) break;
          return size_t(-1);
        }
        done += size_t(w);
      }
      return done;
    };
    if (c.woff < c.wbuf.size()) {
      const size_t w = write_some(c.wbuf.data() + c.woff, c.wbuf.size() - c.woff);
      if (w == size_t(-1)) return false;
      c.woff += w;
      if (c.woff < c.wbuf.size()) return set_out(c, true);
      c.wbuf.clear();
      c.woff = 0;
    }
    // everything nghttp2 has queued (a unary response is three frames: HEADERS, DATA, trailer
    // HEADERS; a drain of many completions is many of them) goes out in ONE send(): one syscall
    // per connection and flush instead of one per frame (tools/host_profile.py: send() was ~45 %
    // of the HTTP/2 workers' CPU)
    bool more = false;  // stopped at the size bound with frames still queued
    for (;;) {
      const uint8_t* p = nullptr;
      const ssize_t len = n.mem_send(c.sess, &p);
      if (len < 0) return false;
      if (len == 0) break;
      c.wbuf.append(reinterpret_cast<const char*>(p), size_t(len));
      if (c.wbuf.size() >= (size_t(1) << 20)) {  // bounded; the rest goes out on EPOLLOUT
        more = true;
        break;
      }
    }
    if (!c.wbuf.empty()) {
      const size_t w = write_some(c.wbuf.data(), c.wbuf.size());
      if (w == size_t(-1)) return false;
      if (w < c.wbuf.size()) {
        c.woff = w;
        return set_out(c, true);
      }
      c.wbuf.clear();
      c.woff = 0;
      if (more) return set_out(c, true);
    }
    if (!n.want_read(c.sess) && !n.want_write(c.sess)) return false;
    return set_out(c, false);
  }
  bool set_out(Conn& c, bool on) {
    if (c.epollout == on) return true;
    epoll_event e{};
    e.events = EPOLLIN | (on ? EPOLLOUT : 0u);
    e.data.u64 = c.id;
    ::epoll_ctl(ep, EPOLL_CTL_MOD, c.fd, &e);
    c.epollout = on;
    return true;
  }

  void close_conn_raw(Conn& c) {
    if (c.sess) ng().session_del(c.sess);
    c.sess = nullptr;
    if (c.fd >= 0) ::close(c.fd);
    c.fd = -1;
  }
  void close_conn(uint64_t id) {
    auto it = conns.find(id);
    if (it == conns.end()) return;
    ::epoll_ctl(ep, EPOLL_CTL_DEL, it->second->fd, nullptr);
    close_conn_raw(*it->second);
    conns.erase(it);
    srv->conns_.fetch_sub(1, std::memory_order_relaxed);
  }

  void dispatch(Conn& c, int32_t sid) {
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) return;
    Stream& st = it->second;
    srv->calls_.fetch_add(1, std::memory_order_relaxed);
    const std::string& d = st.data;
    GrpcReply bad;
    if (d.size() < 5) {
      bad.status = 13;
      bad.message = "grpc: missing message frame";
    } else if (d[0] != 0) {
      bad.status = 12;
      bad.message = "grpc: compressed messages are not supported";
    } else {
      const uint32_t len = (uint32_t(uint8_t(d[1])) << 24) | (uint32_t(uint8_t(d[2])) << 16) |
                           (uint32_t(uint8_t(d[3])) << 8) | uint32_t(uint8_t(d[4]));
      if (size_t(len) + 5 != d.size()) {
        bad.status = 13;
        bad.message = "grpc: message length mismatch";
      }
    }
    if (bad.status) {
      respond(c, sid, bad);
      return;
    }
    const bool hot = srv->hot_.load(std::memory_order_relaxed);
    const uint8_t arpc = hot && srv->router_ ? acct_rpc(st.path) : 0;
    if ((hot && srv->core_ && st.path == kPathTx) || (arpc && srv->router_->serves(arpc))) {
      const uint64_t token = next_token++ & kTokenMask;
      const uint64_t tag = ServeCore::kSinkTag | (uint64_t(idx) << kWorkerShift) | token;
      c.buffered -= std::min(c.buffered, st.data.size());
      Pend& p = pending[token];
      p.conn = c.id;
      p.stream = sid;
      p.path = st.path;
      p.body = std::move(st.data);  // kept for a retry through the cold table
      const char* body = p.body.data() + 5;
      const size_t blen = p.body.size() - 5;
      if (arpc) {
        srv->hot_acct_.fetch_add(1, std::memory_order_relaxed);
        srv->router_->submit(arpc, body, blen, tag, mono_ns());
      } else {
        srv->hot_tx_.fetch_add(1, std::memory_order_relaxed);
        txq.push_back(ServeCore::TxCall{body, blen, tag, mono_ns()});  // handed over after this read
      }
      return;
    }
    c.buffered -= std::min(c.buffered, st.data.size());
    Job j{idx, c.id, sid, st.path, d.substr(5)};
    {
      std::lock_guard<std::mutex> g(srv->jmu_);
      if (hot && st.path == kPathBatch && srv->n_batch_ > 0) {
        srv->hot_batch_.fetch_add(1, std::memory_order_relaxed);
        srv->batch_q_.push_back(std::move(j));
      } else {
        srv->cold_n_.fetch_add(1, std::memory_order_relaxed);
        srv->cold_q_.push_back(std::move(j));
      }
    }
    srv->jcv_.notify_all();
    st.data.clear();
    st.data.shrink_to_fit();
  }

  void respond(Conn& c, int32_t sid, const GrpcReply& r) {
    auto it = c.streams.find(sid);
    if (it == c.streams.end()) return;  // the client reset the stream meanwhile
    Stream& st = it->second;
    const Ng& n = ng();
    static const std::string s200 = "200", ct = "application/grpc";
    if (r.status != 0) {
      srv->errors_.fetch_add(1, std::memory_order_relaxed);
      const std::string code = std::to_string(r.status), msg = pct(r.message);
      const NgNv h[4] = {nv(":status", s200), nv("content-type", ct), nv("grpc-status", code), nv("grpc-message", msg)};
      n.submit_response(c.sess, sid, h, 4, nullptr);  // Trailers-Only
      return;
    }
    st.out.resize(5 + r.body.size());
    const uint32_t len = uint32_t(r.body.size());
    st.out[0] = 0;
    st.out[1] = char(len >> 24);
    st.out[2] = char(len >> 16);
    st.out[3] = char(len >> 8);
    st.out[4] = char(len);
    std::memcpy(&st.out[5], r.body.data(), r.body.size());
    st.off = 0;
    const NgNv h[2] = {nv(":status", s200), nv("content-type", ct)};
    NgDataProvider prd{};
    prd.source.ptr = &st;
    prd.read_callback = read_body;
    n.submit_response(c.sess, sid, h, 2, &prd);
  }

  void drain_done() {
    std::vector<Done> items;
    {
      std::lock_guard<std::mutex> g(qmu);
      items.swap(q);
    }
    std::vector<uint64_t> touched;
    for (Done& d : items) {
      uint64_t cid = d.conn;
      int32_t sid = d.stream;
      if (d.token) {
        auto p = pending.find(d.token);
        if (p == pending.end()) continue;
        cid = p->second.conn;
        sid = p->second.stream;
        if (d.retry) {  // the native path failed: the cold table answers (engine fallback)
          Pend pd = std::move(p->second);
          pending.erase(p);
          // a core failure fails the shard over ("#retry:"); a call no native core serves (the
          // owner has no model core of that kind, or it is stopping) only takes the cold path
          if (!d.cold) srv->note_failure(d.reply.message);
          {
            std::lock_guard<std::mutex> g(srv->jmu_);
            srv->cold_n_.fetch_add(1, std::memory_order_relaxed);
            srv->cold_q_.push_back(
                Job{idx, cid, sid, pd.path + (d.cold ? "#cold:" : "#retry:") + d.reply.message, pd.body.substr(5)});
          }
          srv->jcv_.notify_one();
          continue;
        }
        pending.erase(p);
      }
      auto it = conns.find(cid);
      if (it == conns.end()) continue;
      respond(*it->second, sid, d.reply);
      touched.push_back(cid);
    }
    for (uint64_t cid : touched) {
      auto it = conns.find(cid);
      if (it != conns.end() && !flush(*it->second)) close_conn(cid);
    }
  }
};

// ---------------------------------------------------------------------------- server
GrpcServer::GrpcServer(std::shared_ptr<ServeCore> core, ColdFn cold, int cold_threads, int batch_threads,
                       std::shared_ptr<AcctRouter> router)
    : core_(std::move(core)), router_(std::move(router)), cold_(std::move(cold)), n_cold_(std::max(1, cold_threads)),
      n_batch_(core_ ? std::max(0, batch_threads) : 0) {
  ng();  // fail early without libnghttp2
}

void GrpcServer::note_failure(const std::string& msg) {
  hot_fail_.fetch_add(1, std::memory_order_relaxed);
  std::lock_guard<std::mutex> g(fail_mu_);
  last_failure_ = msg;
}

std::string GrpcServer::last_failure() const {
  std::lock_guard<std::mutex> g(fail_mu_);
  return last_failure_;
}

// completions of hot unary calls (a core's finisher thread): to the worker owning the connection
void GrpcServer::route_done(std::vector<ServeCore::Done>&& outs) {
  thread_local std::vector<std::vector<Worker::Done>> per;  // per worker, posted once per batch
  if (per.size() < workers_.size()) per.resize(workers_.size());
  for (auto& d : outs) {
    const int wi = int((d.tag & ~ServeCore::kSinkTag) >> kWorkerShift);
    if (wi < 0 || size_t(wi) >= workers_.size()) continue;
    Worker::Done w{d.tag & kTokenMask, 0, 0, GrpcReply{}, false};
    if (!d.err.empty()) {
      if (invalid_request(d.err)) {
        w.reply.status = 3;
        w.reply.message = invalid_message(d.err);
      } else {
        w.reply.status = 13;
        w.reply.message = d.err;
        w.retry = true;
        w.cold = d.err.rfind(kColdPrefix, 0) == 0;
      }
    } else {
      w.reply.body = std::move(d.bytes);
    }
    per[size_t(wi)].push_back(std::move(w));
  }
  for (size_t i = 0; i < workers_.size(); ++i) workers_[i]->post_many(per[i]);
}

GrpcServer::~GrpcServer() { stop(); }

int GrpcServer::start(const std::string& host, int port, int workers) {
  if (running_.exchange(true)) throw std::runtime_error("grpc server: already started");
  workers = std::max(1, workers);
  int bound = port;
  for (int i = 0; i < workers; ++i) {
    auto w = std::make_unique<Worker>(this, i);
    w->init(host, bound);
    if (i == 0) bound = w->bound_port();
    workers_.push_back(std::move(w));
  }
  gate_ = std::make_shared<SinkGate>();
  gate_->srv = this;
  // the sink holds the gate, not the server: a finisher that copied it before stop() finds the
  // gate closed (srv null) instead of a destroyed server
  auto sink = [gate = gate_](std::vector<ServeCore::Done>&& outs) {
    std::shared_lock<std::shared_mutex> g(gate->mu);
    if (gate->srv) gate->srv->route_done(std::move(outs));
  };
  if (core_) core_->set_sink(sink);
  if (router_) router_->set_sink(sink);
  for (auto& w : workers_)
    threads_.emplace_back([p = w.get()] {
      name_thread("h2-worker");
      p->run();
    });
  for (int i = 0; i < n_cold_; ++i)
    threads_.emplace_back([this] {
      name_thread("h2-cold");
      cold_loop();
    });
  for (int i = 0; i < n_batch_; ++i)
    threads_.emplace_back([this] {
      name_thread("h2-batch");
      batch_loop();
    });
  return bound;
}

void GrpcServer::stop() {
  if (!running_.exchange(false)) return;
  {
    std::lock_guard<std::mutex> g(jmu_);
    jstop_ = true;
  }
  jcv_.notify_all();
  for (auto& w : workers_) w->stop.store(true);
  if (core_) core_->set_sink(nullptr);
  if (router_) router_->set_sink(nullptr);
  if (gate_) {  // waits for sink calls in progress; later ones (copies taken earlier) see it closed
    std::unique_lock<std::shared_mutex> g(gate_->mu);
    gate_->srv = nullptr;
  }
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  workers_.clear();
}

void GrpcServer::post(int worker, uint64_t conn, int32_t stream, GrpcReply&& r) {
  if (worker < 0 || size_t(worker) >= workers_.size()) return;
  workers_[size_t(worker)]->post(Worker::Done{0, conn, stream, std::move(r), false});
}

void GrpcServer::cold_loop() {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> l(jmu_);
      jcv_.wait(l, [&] { return jstop_ || !cold_q_.empty(); });
      if (cold_q_.empty()) return;
      j = std::move(cold_q_.front());
      cold_q_.pop_front();
    }
    GrpcReply r;
    try {
      r = cold_(j.path, std::move(j.body));
    } catch (const std::exception& e) {
      r.status = 13;
      r.message = e.what();
    }
    post(j.worker, j.conn, j.stream, std::move(r));
  }
}

void GrpcServer::batch_loop() {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> l(jmu_);
      jcv_.wait(l, [&] { return jstop_ || !batch_q_.empty(); });
      if (batch_q_.empty()) return;
      j = std::move(batch_q_.front());
      batch_q_.pop_front();
    }
    GrpcReply r;
    try {
      const std::string_view v = core_->score_batch_view(j.body.data(), j.body.size(), -1, mono_ns());
      r.body.assign(v.data(), v.size());
    } catch (const std::exception& e) {
      if (std::strstr(e.what(), "pb:")) {
        r.status = 3;
        r.message = e.what();
      } else {  // the core failed it: the cold table (engine fallback) answers instead
        note_failure(e.what());
        cold_n_.fetch_add(1, std::memory_order_relaxed);
        try {
          r = cold_(j.path + "#retry:" + e.what(), std::move(j.body));
        } catch (const std::exception& e2) {
          r.status = 13;
          r.message = e2.what();
        }
      }
    }
    post(j.worker, j.conn, j.stream, std::move(r));
  }
}

GrpcServer::Stats GrpcServer::stats() const {
  return Stats{calls_.load(), hot_tx_.load(), hot_batch_.load(), cold_n_.load(), errors_.load(), conns_.load(),
               hot_acct_.load(), hot_fail_.load()};
}

// ---------------------------------------------------------------------------- load generator
// Open-loop unary gRPC load over `conns` HTTP/2 connections (one thread each): calls are issued
// on a fixed schedule (rate / conns per connection) whatever the server's pace, up to
// max_inflight per connection; latency counts from the SCHEDULED send time, so a server that
// falls behind shows growing latency, not a lower offered load (tools/bench_e2e.py
// --client native: the Python clients topped out before the native server did).
namespace {

struct LoadConn {
  struct Call {
    int64_t t_sched;
    std::string body;  // 5-byte prefix + message
    size_t off = 0;
    int status = -1;
  };
  void* sess = nullptr;
  std::unordered_map<int32_t, std::unique_ptr<Call>> calls;  // heap calls: the providers point at them
  std::vector<double>* lat = nullptr;
  std::vector<double>* sched = nullptr;
  int64_t t0 = 0;
  int64_t* errors = nullptr;
  int64_t* done = nullptr;
  int64_t* last = nullptr;  // latest completion (mono ns)

  static ssize_t read_req(void*, int32_t, uint8_t* buf, size_t len, uint32_t* flags, NgDataSource* src, void*) {
    auto* c = static_cast<Call*>(src->ptr);
    const size_t n = std::min(len, c->body.size() - c->off);
    std::memcpy(buf, c->body.data() + c->off, n);
    c->off += n;
    if (c->off == c->body.size()) *flags |= kDataEof;
    return ssize_t(n);
  }
  static int on_header(void*, const void* frame, const uint8_t* name, size_t namelen, const uint8_t* value,
                       size_t valuelen, uint8_t, void* ud) {
    auto* lc = static_cast<LoadConn*>(ud);
    const auto* hd = static_cast<const NgFrameHd*>(frame);
    if (namelen == 11 && std::memcmp(name, "grpc-status", 11) == 0) {
      auto it = lc->calls.find(hd->stream_id);
      if (it != lc->calls.end()) it->second->status = std::atoi(std::string(reinterpret_cast<const char*>(value), valuelen).c_str());
    }
    return 0;
  }
  static int on_close(void*, int32_t sid, uint32_t err, void* ud) {
    auto* lc = static_cast<LoadConn*>(ud);
    auto it = lc->calls.find(sid);
    if (it == lc->calls.end()) return 0;
    const int64_t t = mono_ns();
    if (t > *lc->last) *lc->last = t;
    if (err == 0 && it->second->status == 0) {
      lc->lat->push_back(double(t - it->second->t_sched) * 1e-6);
      lc->sched->push_back(double(it->second->t_sched - lc->t0) * 1e-6);
    } else {
      ++*lc->errors;
    }
    ++*lc->done;
    lc->calls.erase(it);
    return 0;
  }
};

}  // namespace

LoadResult grpc_load(const std::string& host, int port, const std::string& path, const std::vector<std::string>& payloads,
                     double rate, double seconds, int conns, int max_inflight) {
  const Ng& n = ng();
  if (payloads.empty() || rate <= 0 || conns < 1) throw std::runtime_error("grpc_load: arguments");
  LoadResult out;
  std::vector<std::vector<double>> lats(static_cast<size_t>(conns)), scheds(static_cast<size_t>(conns));
  std::vector<int64_t> errs(static_cast<size_t>(conns), 0), sent(static_cast<size_t>(conns), 0),
      done(static_cast<size_t>(conns), 0), last(static_cast<size_t>(conns), 0);
  std::vector<std::string> frames(payloads.size());
  for (size_t i = 0; i < payloads.size(); ++i) {
    const uint32_t len = uint32_t(payloads[i].size());
    std::string f(5, '\0');
    f[1] = char(len >> 24); f[2] = char(len >> 16); f[3] = char(len >> 8); f[4] = char(len);
    frames[i] = f + payloads[i];
  }
  const std::string authority = host + ":" + std::to_string(port);
  const int64_t t0 = mono_ns() + 200000000;  // 200 ms for the connections to come up (HTTP/2 preface, settings)
  const int64_t t_end = t0 + int64_t(seconds * 1e9);
  std::vector<std::thread> th;
  std::atomic<int> failed{0};
  for (int ci = 0; ci < conns; ++ci) {
    th.emplace_back([&, ci] {
      name_thread("h2-loadgen");
      const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons(uint16_t(port));
      ::inet_pton(AF_INET, host == "localhost" ? "127.0.0.1" : host.c_str(), &a.sin_addr);
      if (fd < 0 || ::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
        failed.fetch_add(1);
        if (fd >= 0) ::close(fd);
        return;
      }
      int one = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL) | O_NONBLOCK);
      void* cbs = nullptr;
      n.callbacks_new(&cbs);
      n.set_on_header(cbs, LoadConn::on_header);
      n.set_on_stream_close(cbs, LoadConn::on_close);
      LoadConn lc;
      lc.lat = &lats[size_t(ci)];
      lc.sched = &scheds[size_t(ci)];
      lc.t0 = t0;
      lc.errors = &errs[size_t(ci)];
      lc.done = &done[size_t(ci)];
      lc.last = &last[size_t(ci)];
      n.client_new(&lc.sess, cbs, &lc);
      n.callbacks_del(cbs);
      const NgSettingsEntry iv[2] = {{kSettingsMaxStreams, 100000}, {kSettingsInitialWindow, 8u << 20}};
      n.submit_settings(lc.sess, 0, iv, 2);
      const double interval = double(conns) / rate * 1e9;  // ns between this connection's calls
      int64_t k = 0;
      std::vector<char> rbuf(size_t(256) << 10);
      std::string wpend;
      static const std::string post = "POST", scheme = "http", ct = "application/grpc", te = "trailers";
      bool ok = true;
      while (ok) {
        const int64_t now = mono_ns();
        if (now > t_end + 10000000000LL) break;  // 10 s grace for stragglers
        // issue every call whose scheduled time has come
        while (true) {
          const int64_t ts = t0 + int64_t(double(k) * interval) + int64_t(double(ci) * interval / conns);
          if (ts > now || ts >= t_end) break;
          if (int(lc.calls.size()) >= max_inflight) break;
          auto c = std::make_unique<LoadConn::Call>();
          c->t_sched = ts;
          c->body = frames[size_t((k * conns + ci) % int64_t(frames.size()))];
          const NgNv h[6] = {nv(":method", post), nv(":scheme", scheme), nv(":path", path),
                             nv(":authority", authority), nv("content-type", ct), nv("te", te)};
          NgDataProvider prd{};
          prd.read_callback = LoadConn::read_req;
          prd.source.ptr = c.get();
          const int32_t sid = n.submit_request(lc.sess, nullptr, h, 6, &prd, nullptr);
          ++k;
          if (sid < 0) {
            ++errs[size_t(ci)];
            continue;
          }
          lc.calls.emplace(sid, std::move(c));
          ++sent[size_t(ci)];
        }
        const uint8_t* p = nullptr;
        for (;;) {
          const ssize_t len = n.mem_send(lc.sess, &p);
          if (len <= 0) break;
          wpend.append(reinterpret_cast<const char*>(p), size_t(len));
        }
        while (!wpend.empty()) {
          const ssize_t w = ::send(fd, wpend.data(), wpend.size(), MSG_NOSIGNAL);
          if (w < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK) break;
            ok = false;
            break;
          }
          wpend.erase(0, size_t(w));
        }
        const ssize_t r = ::recv(fd, rbuf.data(), rbuf.size(), 0);
        if (r > 0) {
          if (n.mem_recv(lc.sess, reinterpret_cast<const uint8_t*>(rbuf.data()), size_t(r)) < 0) ok = false;
        } else if (r == 0) {
          ok = false;
        } else if (errno != EAGAIN && errno != EWOULDBLOCK) {
          ok = false;
        } else {
          if (now >= t_end && lc.calls.empty()) break;
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
      }
      errs[size_t(ci)] += int64_t(lc.calls.size());  // unanswered at the end
      n.session_del(lc.sess);
      ::close(fd);
    });
  }
  for (auto& t : th) t.join();
  for (int ci = 0; ci < conns; ++ci) {
    out.latency_ms.insert(out.latency_ms.end(), lats[size_t(ci)].begin(), lats[size_t(ci)].end());
    out.sched_ms.insert(out.sched_ms.end(), scheds[size_t(ci)].begin(), scheds[size_t(ci)].end());
    out.errors += errs[size_t(ci)];
    out.sent += sent[size_t(ci)];
  }
  out.errors += int64_t(failed.load()) * int64_t(rate * seconds / conns);
  out.seconds = seconds;
  int64_t lastc = t0;
  for (int64_t v : last) lastc = std::max(lastc, v);
  out.elapsed = std::max(seconds, double(lastc - t0) * 1e-9);
  return out;
}

}  // namespace igp
