// mlcomp-broker: the framework's task-queue daemon (replaces the vendored redis-server
// + Celery of the reference, mlcomp/bin/redis-server, mlcomp/worker/app.py).
//
// Single-threaded epoll server speaking a line protocol (one request, one response):
//   PUSH <queue> <json>            -> OK <id>
//   POP <timeout_ms> <q1> [q2 ...] -> MSG <queue> <id> <json> | NIL      (blocking, leased)
//   ACK <id> | NACK <id>           -> OK 1 | OK 0 (1: the lease existed; NACK: back to the head
//                                                   of its queue)
//   REVOKE <id>                    -> OK 1 | OK 0 (drop a pending message)
//   HAS <id>                       -> OK 1 | OK 0 (the message is queued or leased)
//   SET <key> <json>               -> OK          (result store)
//   GET <key> <timeout_ms>         -> VAL <json> | NIL (blocking, consumes the value)
//   LEN <queue>                    -> OK <n>
//   PING                           -> PONG
//   STATS                          -> OK {"queues":..,"leased":..,"results":..,"clients":..}
// A leased message whose consumer disconnects before ACK is re-queued at the head of
// its queue (and handed to a blocked POP waiter right away), so a crashed worker never
// loses a task.  Waiters are served FIFO.  Requests a client sent before half-closing
// its socket are still executed and answered (the connection closes once its replies,
// including a blocked POP/GET's, have been written).
//
// --journal <file>: every PUSH / ACK / REVOKE is appended to the file before it is
// answered, and a restarted broker replays it: messages pushed and not yet acked or
// revoked (leased ones included) are queued again in id order, so a broker restart does
// not orphan dispatched tasks.  The journal is rewritten to the live set at start-up and
// whenever it grows past 4x that set.  It survives a crash of the broker process (the
// writes are flushed to the kernel), not a power loss (no fsync).
//
// usage: mlcomp-broker [--host 127.0.0.1] [--port 6380] [--journal FILE] [--compact-every N]
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

struct Msg {
  std::string id, queue, payload;
};

struct Conn;

struct Waiter {  // a blocked POP or GET
  Conn* conn;
  bool is_pop;
  std::vector<std::string> keys;  // queues (POP) or one result key (GET)
  Clock::time_point deadline;
};

struct Conn {
  int fd;
  std::string in, out;
  bool waiting = false;
  std::list<Waiter>::iterator wit;
  std::vector<std::string> leased;  // message ids leased to this connection
  bool closed = false;
  bool eof = false;                 // the peer half-closed: close once the replies are out
};

class Broker {
 public:
  explicit Broker(int listen_fd) : lfd_(listen_fd) {}
  ~Broker() {
    for (auto& kv : conns_) close(kv.first);
    if (ep_ >= 0) close(ep_);
    close(lfd_);
    if (jf_) fclose(jf_);
  }
  bool open_journal(const std::string& path);
  void run();

 private:
  int lfd_, ep_ = -1;
  unsigned long long next_id_ = 1;
  std::unordered_map<std::string, std::deque<Msg>> queues_;
  std::unordered_map<std::string, Msg> leased_;
  std::unordered_map<std::string, std::string> results_;
  std::unordered_map<int, std::unique_ptr<Conn>> conns_;
  std::list<Waiter> waiters_;
  std::unordered_set<std::string> queued_ids_;   // ids in queues_ (HAS without a scan)
  bool need_wake_ = false;  // set by close_conn (re-queued leases); drained by run()
  std::string jpath_;
  FILE* jf_ = nullptr;
  size_t jlines_ = 0;
 public:
  size_t compact_every_ = 0;   // --compact-every N (tests): compact whenever N lines accrued
 private:

  void journal(const char* tag, const std::string& id, const Msg* m = nullptr);
  void compact_journal();
  void enqueue_front(const Msg& m) { queues_[m.queue].push_front(m); queued_ids_.insert(m.id); }

  void accept_all();
  void on_read(Conn* c);
  void flush(Conn* c);
  void close_conn(Conn* c);
  void handle(Conn* c, const std::string& line);
  void reply(Conn* c, const std::string& s) { c->out += s; c->out += '\n'; }
  bool try_pop(Conn* c, const std::vector<std::string>& qs);
  bool try_get(Conn* c, const std::string& key);
  void wake();
  void expire();
  int next_timeout_ms();
  void watch_write(Conn* c, bool on);
};

std::vector<std::string> split(const std::string& s, size_t max_parts) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < s.size() && out.size() + 1 < max_parts) {
    while (i < s.size() && s[i] == ' ') ++i;
    if (i >= s.size()) break;
    size_t j = s.find(' ', i);
    if (j == std::string::npos) j = s.size();
    out.push_back(s.substr(i, j - i));
    i = j;
  }
  while (i < s.size() && s[i] == ' ') ++i;
  if (i < s.size()) out.push_back(s.substr(i));
  return out;
}

void set_nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL, 0) | O_NONBLOCK); }

void Broker::watch_write(Conn* c, bool on) {
  epoll_event ev{};
  // after EOF the read side stays readable forever: stop watching it (no busy loop while
  // a half-closed client's POP/GET is still blocked)
  ev.events = (c->eof ? 0u : (uint32_t)(EPOLLIN | EPOLLRDHUP)) | (on ? EPOLLOUT : 0u);
  ev.data.fd = c->fd;
  epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &ev);
}

void Broker::accept_all() {
  for (;;) {
    int fd = accept(lfd_, nullptr, nullptr);
    if (fd < 0) return;
    set_nonblock(fd);
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    auto c = std::make_unique<Conn>();
    c->fd = fd;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLRDHUP;
    ev.data.fd = fd;
    epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
    conns_[fd] = std::move(c);
  }
}

void Broker::close_conn(Conn* c) {
  if (c->closed) return;
  c->closed = true;
  if (c->waiting) { waiters_.erase(c->wit); c->waiting = false; }
  // re-queue leased messages at the head of their queues (newest first keeps order)
  for (auto it = c->leased.rbegin(); it != c->leased.rend(); ++it) {
    auto l = leased_.find(*it);
    if (l == leased_.end()) continue;
    enqueue_front(l->second);
    leased_.erase(l);
    need_wake_ = true;
  }
  // waiters are woken from run(), not here: close_conn can be reached from flush()
  // inside wake(), whose iterator a nested wake() would invalidate
  epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
}

void Broker::flush(Conn* c) {
  if (c->closed) return;
  while (!c->out.empty()) {
    ssize_t n = send(c->fd, c->out.data(), c->out.size(), MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) { watch_write(c, true); return; }
      close_conn(c);
      return;
    }
    c->out.erase(0, (size_t)n);
  }
  if (c->eof && !c->waiting) { close_conn(c); return; }
  watch_write(c, false);
}

bool Broker::try_pop(Conn* c, const std::vector<std::string>& qs) {
  for (const auto& q : qs) {
    auto it = queues_.find(q);
    if (it == queues_.end() || it->second.empty()) continue;
    Msg m = it->second.front();
    it->second.pop_front();
    queued_ids_.erase(m.id);
    reply(c, "MSG " + q + " " + m.id + " " + m.payload);
    c->leased.push_back(m.id);
    leased_[m.id] = m;
    return true;
  }
  return false;
}

bool Broker::try_get(Conn* c, const std::string& key) {
  auto it = results_.find(key);
  if (it == results_.end()) return false;
  reply(c, "VAL " + it->second);
  results_.erase(it);
  return true;
}

void Broker::wake() {
  for (auto it = waiters_.begin(); it != waiters_.end();) {
    Conn* c = it->conn;
    bool done = it->is_pop ? try_pop(c, it->keys) : try_get(c, it->keys[0]);
    if (done) {
      c->waiting = false;
      it = waiters_.erase(it);
      flush(c);
    } else {
      ++it;
    }
  }
}

void Broker::expire() {
  auto now = Clock::now();
  for (auto it = waiters_.begin(); it != waiters_.end();) {
    if (it->deadline <= now) {
      Conn* c = it->conn;
      c->waiting = false;
      reply(c, "NIL");
      it = waiters_.erase(it);
      flush(c);
    } else {
      ++it;
    }
  }
}

int Broker::next_timeout_ms() {
  if (waiters_.empty()) return 1000;
  auto now = Clock::now();
  long best = 1000;
  for (auto& w : waiters_) {
    long ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(w.deadline - now).count();
    if (ms < best) best = ms;
  }
  return best < 0 ? 0 : (int)best;
}

void Broker::handle(Conn* c, const std::string& line) {
  if (line.empty()) return;
  auto sp = line.find(' ');
  std::string cmd = line.substr(0, sp);
  std::string rest = sp == std::string::npos ? "" : line.substr(sp + 1);
  if (cmd == "PING") { reply(c, "PONG"); return; }
  if (cmd == "PUSH") {
    auto a = split(rest, 2);
    if (a.size() < 2) { reply(c, "ERR usage: PUSH queue payload"); return; }
    Msg m{std::to_string(next_id_++), a[0], a[1]};
    // state first, journal after: a compaction triggered by this line rewrites the
    // journal from the live state, which must already hold the message
    queues_[a[0]].push_back(m);
    queued_ids_.insert(m.id);
    journal("P", m.id, &m);
    reply(c, "OK " + m.id);
    wake();
    return;
  }
  if (cmd == "POP") {
    auto a = split(rest, 1 << 20);
    if (a.size() < 2) { reply(c, "ERR usage: POP timeout_ms queue..."); return; }
    long ms = atol(a[0].c_str());
    std::vector<std::string> qs(a.begin() + 1, a.end());
    if (try_pop(c, qs)) return;
    if (ms <= 0) { reply(c, "NIL"); return; }
    waiters_.push_back(Waiter{c, true, qs, Clock::now() + std::chrono::milliseconds(ms)});
    c->waiting = true;
    c->wit = std::prev(waiters_.end());
    return;
  }
  if (cmd == "ACK" || cmd == "NACK") {
    auto l = leased_.find(rest);
    const bool had = l != leased_.end();
    if (had) {
      if (cmd == "NACK") enqueue_front(l->second);
      leased_.erase(l);
      for (auto& kv : conns_) {
        auto& v = kv.second->leased;
        for (auto it = v.begin(); it != v.end(); ++it)
          if (*it == rest) { v.erase(it); break; }
      }
      // after the lease is gone: a compaction at this line must not write it back as live
      if (cmd == "ACK") journal("A", rest);
    }
    reply(c, had ? "OK 1" : "OK 0");
    if (cmd == "NACK") wake();
    return;
  }
  if (cmd == "REVOKE") {
    if (queued_ids_.count(rest)) {
      for (auto& kv : queues_) {
        auto& dq = kv.second;
        for (auto it = dq.begin(); it != dq.end(); ++it)
          if (it->id == rest) {
            dq.erase(it);
            queued_ids_.erase(rest);
            journal("R", rest);
            reply(c, "OK 1");
            return;
          }
      }
    }
    reply(c, "OK 0");
    return;
  }
  if (cmd == "HAS") {
    reply(c, (queued_ids_.count(rest) || leased_.count(rest)) ? "OK 1" : "OK 0");
    return;
  }
  if (cmd == "SET") {
    auto a = split(rest, 2);
    if (a.size() < 2) { reply(c, "ERR usage: SET key payload"); return; }
    results_[a[0]] = a[1];
    reply(c, "OK");
    wake();
    return;
  }
  if (cmd == "GET") {
    auto a = split(rest, 2);
    if (a.empty()) { reply(c, "ERR usage: GET key [timeout_ms]"); return; }
    long ms = a.size() > 1 ? atol(a[1].c_str()) : 0;
    if (try_get(c, a[0])) return;
    if (ms <= 0) { reply(c, "NIL"); return; }
    waiters_.push_back(Waiter{c, false, {a[0]}, Clock::now() + std::chrono::milliseconds(ms)});
    c->waiting = true;
    c->wit = std::prev(waiters_.end());
    return;
  }
  if (cmd == "LEN") {
    auto it = queues_.find(rest);
    reply(c, "OK " + std::to_string(it == queues_.end() ? 0 : it->second.size()));
    return;
  }
  if (cmd == "STATS") {
    std::string s = "OK {\"queues\":{";
    bool first = true;
    for (auto& kv : queues_) {
      if (kv.second.empty()) continue;
      if (!first) s += ",";
      first = false;
      s += "\"" + kv.first + "\":" + std::to_string(kv.second.size());
    }
    s += "},\"leased\":" + std::to_string(leased_.size()) + ",\"results\":" +
         std::to_string(results_.size()) + ",\"clients\":" + std::to_string(conns_.size()) + "}";
    reply(c, s);
    return;
  }
  reply(c, "ERR unknown command " + cmd);
}

void Broker::on_read(Conn* c) {
  char buf[65536];
  bool eof = false;
  for (;;) {
    ssize_t n = recv(c->fd, buf, sizeof(buf), 0);
    if (n > 0) { c->in.append(buf, (size_t)n); continue; }
    if (n == 0) { eof = true; break; }  // peer half-closed: serve what it sent first
    if (errno == EAGAIN || errno == EWOULDBLOCK) break;
    close_conn(c);
    return;
  }
  size_t pos;
  // one outstanding blocking request per connection: stop parsing while waiting
  while (!c->waiting && (pos = c->in.find('\n')) != std::string::npos) {
    std::string line = c->in.substr(0, pos);
    if (!line.empty() && line.back() == '\r') line.pop_back();
    c->in.erase(0, pos + 1);
    handle(c, line);
  }
  if (c->in.size() > (64u << 20)) { close_conn(c); return; }
  if (eof && !c->eof) {
    c->eof = true;
    // the requests still buffered behind a blocked one are dropped with the connection:
    // a half-closed client has stopped sending, but is owed the replies already due
    if (!c->waiting) c->in.clear();
  }
  flush(c);   // closes a half-closed connection once nothing is pending
}

void Broker::journal(const char* tag, const std::string& id, const Msg* m) {
  if (!jf_) return;
  if (m)
    fprintf(jf_, "%s %s %s %s\n", tag, id.c_str(), m->queue.c_str(), m->payload.c_str());
  else
    fprintf(jf_, "%s %s\n", tag, id.c_str());
  fflush(jf_);
  ++jlines_;
  if (compact_every_ ? jlines_ >= compact_every_
                     : jlines_ > 10000 && jlines_ > 4 * (queued_ids_.size() + leased_.size()))
    compact_journal();
}

// rewrite the journal to the live set (queued + leased, in id order) via tmp + rename
void Broker::compact_journal() {
  std::vector<const Msg*> live;
  for (auto& kv : queues_)
    for (auto& m : kv.second) live.push_back(&m);
  for (auto& kv : leased_) live.push_back(&kv.second);
  std::sort(live.begin(), live.end(), [](const Msg* a, const Msg* b) {
    return std::stoull(a->id) < std::stoull(b->id);
  });
  const std::string tmp = jpath_ + ".tmp";
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) { perror("journal compaction"); return; }
  for (const Msg* m : live) fprintf(f, "P %s %s %s\n", m->id.c_str(), m->queue.c_str(), m->payload.c_str());
  fclose(f);
  if (rename(tmp.c_str(), jpath_.c_str()) != 0) { perror("journal rename"); return; }
  if (jf_) fclose(jf_);
  jf_ = fopen(jpath_.c_str(), "a");
  jlines_ = live.size();
}

// replay: P adds, A / R remove; survivors are queued in id order
bool Broker::open_journal(const std::string& path) {
  jpath_ = path;
  std::map<unsigned long long, Msg> live;
  if (FILE* f = fopen(path.c_str(), "r")) {
    std::string line;
    int ch;
    for (;;) {
      line.clear();
      while ((ch = fgetc(f)) != EOF && ch != '\n') line.push_back((char)ch);
      if (line.empty() && ch == EOF) break;
      auto a = split(line, 4);
      if (a.size() >= 2) {
        unsigned long long id = strtoull(a[1].c_str(), nullptr, 10);
        if (a[0] == "P" && a.size() == 4) live[id] = Msg{a[1], a[2], a[3]};
        else if (a[0] == "A" || a[0] == "R") live.erase(id);
        if (id >= next_id_) next_id_ = id + 1;
      }
      if (ch == EOF) break;
    }
    fclose(f);
  }
  for (auto& kv : live) {
    queues_[kv.second.queue].push_back(kv.second);
    queued_ids_.insert(kv.second.id);
  }
  compact_journal();
  if (!jf_) return false;
  fprintf(stdout, "mlcomp-broker journal %s: %zu pending message(s) restored\n", path.c_str(), live.size());
  return true;
}

// SIGTERM / SIGINT end the event loop so the broker exits through its destructors (a
// clean shutdown is what lets the ASan/LSan build report real leaks, not killed state)
volatile sig_atomic_t g_stop = 0;
void on_stop_signal(int) { g_stop = 1; }

void Broker::run() {
  ep_ = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd_;
  epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &ev);
  std::vector<epoll_event> events(256);
  while (!g_stop) {
    int n = epoll_wait(ep_, events.data(), (int)events.size(), next_timeout_ms());
    if (n < 0 && errno != EINTR) { perror("epoll_wait"); return; }
    if (g_stop) break;
    for (int i = 0; i < n; ++i) {
      int fd = events[i].data.fd;
      if (fd == lfd_) { accept_all(); continue; }
      auto it = conns_.find(fd);
      if (it == conns_.end()) continue;
      Conn* c = it->second.get();
      if (events[i].events & EPOLLERR) { close_conn(c); continue; }
      // both directions gone: nobody can read a reply any more
      if (c->eof && (events[i].events & EPOLLHUP)) { close_conn(c); continue; }
      // EPOLLIN / EPOLLRDHUP / EPOLLHUP: read to EOF (on_read parses and answers the
      // complete requests still buffered, then closes)
      if (events[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP)) on_read(c);
      if (!c->closed && (events[i].events & EPOLLOUT)) flush(c);
    }
    while (need_wake_) { need_wake_ = false; wake(); }
    expire();
    // a waiter that got its answer may have more pipelined requests queued
    for (auto it = conns_.begin(); it != conns_.end();) {
      Conn* c = it->second.get();
      if (c->closed) { it = conns_.erase(it); continue; }
      if (!c->waiting && !c->eof && c->in.find('\n') != std::string::npos) on_read(c);
      ++it;
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::string host = "127.0.0.1", jpath;
  int port = 6380;
  long compact_every = 0;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--host")) host = argv[i + 1];
    else if (!strcmp(argv[i], "--port")) port = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "--journal")) jpath = argv[i + 1];
    else if (!strcmp(argv[i], "--compact-every")) compact_every = atol(argv[i + 1]);
  }
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa{};
  sa.sa_handler = on_stop_signal;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = 0;                    // no SA_RESTART: epoll_wait returns EINTR
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    fprintf(stderr, "bad host %s\n", host.c_str());
    return 2;
  }
  if (bind(lfd, (sockaddr*)&addr, sizeof(addr)) < 0) { perror("bind"); return 1; }
  if (listen(lfd, 512) < 0) { perror("listen"); return 1; }
  set_nonblock(lfd);
  Broker broker(lfd);
  broker.compact_every_ = compact_every > 0 ? (size_t)compact_every : 0;
  if (!jpath.empty() && !broker.open_journal(jpath)) {
    fprintf(stderr, "cannot open journal %s\n", jpath.c_str());
    return 1;
  }
  fprintf(stdout, "mlcomp-broker listening on %s:%d\n", host.c_str(), port);
  fflush(stdout);
  broker.run();
  return 0;
}
