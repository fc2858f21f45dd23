// mlcomp_amd native input pipeline: record files + a threaded batch gatherer.
//
// The reference feeds Catalyst from a PyTorch DataLoader (python workers decoding images,
// `mlcomp/contrib/dataset/classify.py:16-138`).  At ~11.5k img/s per MI355X (92k img/s per
// 8-GPU node) a python pipeline is the bottleneck, so the MI355X design splits the work:
//   * host (this file): a memory-mapped record file of fixed-size uint8 HWC images + int32
//     labels; per epoch a seeded global shuffle, sharded by rank; worker threads copy the
//     raw records of a batch into a caller-owned (pinned) slot and draw the per-sample
//     augmentation parameters (RandomResizedCrop box + horizontal flip, or the centre crop
//     for evaluation) from a counter-based RNG keyed by (seed, epoch, sample);
//   * device (csrc/kernels/augment.hip): one kernel crops, bilinearly resizes, flips,
//     normalises and writes the layout the model's first layer reads (the native stem's
//     space-to-depth image), so the host never touches a float and PCIe carries uint8.
//
// File format (".mlrec", little endian): 64-byte header
//   char magic[8] = "MLREC001"; u32 H, W, C; u32 label_bytes (= 4); u64 count;
//   u64 record_bytes (= H*W*C + 4); u8 reserved[24]
// followed by `count` records {u8 image[H][W][C]; i32 label}.
//
// Slot protocol: the caller registers `depth` slots (image buffer of batch*H*W*C bytes,
// int64 labels[batch], int32 params[batch][5]); next() blocks until the next batch of the
// epoch (in order) is complete and returns its slot, release(slot) hands it back.  Batches
// are split into chunks of samples so every worker thread helps fill the batch the
// consumer waits for.  All shared state is guarded by one mutex; the copies run unlocked.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

namespace {

constexpr char MAGIC[8] = {'M', 'L', 'R', 'E', 'C', '0', '0', '1'};

struct Header {
  char magic[8];
  uint32_t H, W, C, label_bytes;
  uint64_t count, record_bytes;
  uint8_t reserved[24];
};
static_assert(sizeof(Header) == 64, "header layout");

struct RecordFile {
  int fd = -1;
  const uint8_t* map = nullptr;
  size_t size = 0;
  Header h{};
  const uint8_t* record(uint64_t i) const { return map + sizeof(Header) + i * h.record_bytes; }
};

// counter-based RNG: splitmix64 of a key, so a sample's augmentation depends only on
// (seed, epoch, sample index) - not on thread scheduling
inline uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t key) : s(mix(key)) {}
  uint64_t next() { return s = mix(s); }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

enum SlotState { FREE = 0, FILLING = 1, READY = 2, INUSE = 3 };

struct Slot {
  uint8_t* img = nullptr;
  int64_t* lab = nullptr;
  int32_t* par = nullptr;
  SlotState state = FREE;
  int64_t batch = -1;
  int remaining = 0;   // chunks still being filled
};

struct Loader {
  const RecordFile* rf;
  int batch, out_h, out_w, train;
  double smin, smax, rmin, rmax;
  uint64_t seed;
  int rank, world, shuffle, drop_last;
  int chunk = 16;
  std::vector<Slot> slots;
  // epoch
  uint64_t epoch = 0;
  std::vector<uint64_t> order;   // this rank's samples, padded to a whole number of batches
  int64_t nbatches = 0, nitems = 0, next_item = 0, consume_next = 0;
  int filling = 0;               // chunks being copied right now
  bool started = false, stop = false;
  std::mutex mu;
  std::condition_variable cv_work, cv_ready, cv_idle;
  std::vector<std::thread> workers;

  int chunks_per_batch() const { return (batch + chunk - 1) / chunk; }

  // one sample's augmentation: {y0, x0, h, w, flip} of the source box
  void params(uint64_t sample, int32_t* p) const {
    const int H = (int)rf->h.H, W = (int)rf->h.W;
    Rng g(seed * 0x100000001b3ull ^ (epoch << 40) ^ sample);
    if (!train) {   // centre crop of the output size (whole image if it is smaller)
      const int h = std::min(H, out_h), w = std::min(W, out_w);
      p[0] = (H - h) / 2; p[1] = (W - w) / 2; p[2] = h; p[3] = w; p[4] = 0;
      return;
    }
    const double area = (double)H * W;
    for (int attempt = 0; attempt < 10; ++attempt) {   // torchvision RandomResizedCrop
      const double a = area * (smin + (smax - smin) * g.uniform());
      const double lr = std::log(rmin) + (std::log(rmax) - std::log(rmin)) * g.uniform();
      const double r = std::exp(lr);
      const int w = (int)std::lround(std::sqrt(a * r)), h = (int)std::lround(std::sqrt(a / r));
      if (w > 0 && h > 0 && w <= W && h <= H) {
        p[0] = (int)(g.next() % (uint64_t)(H - h + 1));
        p[1] = (int)(g.next() % (uint64_t)(W - w + 1));
        p[2] = h; p[3] = w; p[4] = (int)(g.next() & 1);
        return;
      }
    }
    const int s = std::min(H, W);   // fallback: centre square
    p[0] = (H - s) / 2; p[1] = (W - s) / 2; p[2] = s; p[3] = s; p[4] = (int)(g.next() & 1);
  }

  void fill(Slot& sl, int64_t b, int c) {
    const size_t ib = (size_t)rf->h.H * rf->h.W * rf->h.C;
    const int i0 = c * chunk, i1 = std::min(batch, i0 + chunk);
    for (int i = i0; i < i1; ++i) {
      const uint64_t s = order[(size_t)b * batch + i];
      const uint8_t* rec = rf->record(s);
      std::memcpy(sl.img + (size_t)i * ib, rec, ib);
      int32_t lab;
      std::memcpy(&lab, rec + ib, 4);
      sl.lab[i] = lab;
      params(s, sl.par + 5 * i);
    }
  }

  void worker() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv_work.wait(lk, [&] { return stop || (started && next_item < nitems); });
      if (stop) return;
      const int64_t item = next_item;
      const int64_t b = item / chunks_per_batch();
      const int c = (int)(item % chunks_per_batch());
      Slot& sl = slots[(size_t)(b % (int64_t)slots.size())];
      if (!(sl.batch == b && sl.state == FILLING) && sl.state != FREE) {
        // the slot still holds an older batch: wait for the consumer to release it
        cv_work.wait(lk, [&] { return stop || !started || next_item != item || sl.state == FREE ||
                                      (sl.batch == b && sl.state == FILLING); });
        continue;
      }
      if (sl.state == FREE) { sl.state = FILLING; sl.batch = b; sl.remaining = chunks_per_batch(); }
      ++next_item;
      ++filling;
      lk.unlock();
      fill(sl, b, c);
      lk.lock();
      --filling;
      if (--sl.remaining == 0) { sl.state = READY; cv_ready.notify_all(); }
      if (filling == 0) cv_idle.notify_all();
      cv_work.notify_all();
    }
  }

  void start_epoch(uint64_t e) {
    std::unique_lock<std::mutex> lk(mu);
    // stop claiming new work of the old epoch, let the copies in flight finish
    next_item = nitems;
    cv_idle.wait(lk, [&] { return filling == 0; });
    for (auto& s : slots) { s.state = FREE; s.batch = -1; s.remaining = 0; }
    epoch = e;
    const uint64_t n = rf->h.count;
    std::vector<uint64_t> all(n);
    std::iota(all.begin(), all.end(), 0ull);
    if (shuffle) {   // Fisher-Yates with the epoch's RNG: identical on every rank
      Rng g(seed ^ 0x5851f42d4c957f2dull ^ (e * 0x2545f4914f6cdd1dull));
      for (uint64_t i = n; i > 1; --i) std::swap(all[i - 1], all[g.next() % i]);
    }
    // shard: pad to a multiple of world (wrapping), rank takes every world-th sample
    const uint64_t per = (n + world - 1) / world;
    order.clear();
    for (uint64_t i = 0; i < per; ++i) order.push_back(all[(i * world + rank) % n]);
    const uint64_t nb = drop_last ? per / batch : (per + batch - 1) / batch;
    // a last partial batch is filled up by wrapping around this rank's samples (fixed slot
    // shape); RecordLoader.real_rows() tells the consumer how many rows are real
    for (uint64_t i = order.size(); i < nb * batch; ++i) order.push_back(order[i % per]);
    nbatches = (int64_t)nb;
    nitems = nbatches * chunks_per_batch();
    next_item = 0;
    consume_next = 0;
    started = true;
    cv_work.notify_all();
  }

  int next(int64_t* batch_index) {
    std::unique_lock<std::mutex> lk(mu);
    if (!started || consume_next >= nbatches) return -1;
    const int64_t b = consume_next;
    Slot& sl = slots[(size_t)(b % (int64_t)slots.size())];
    cv_ready.wait(lk, [&] { return stop || (sl.batch == b && sl.state == READY); });
    if (stop) return -1;
    sl.state = INUSE;
    ++consume_next;
    if (batch_index) *batch_index = b;
    return (int)(b % (int64_t)slots.size());
  }

  void release(int s) {
    std::lock_guard<std::mutex> lk(mu);
    if (s < 0 || s >= (int)slots.size() || slots[(size_t)s].state != INUSE) return;
    slots[(size_t)s].state = FREE;
    slots[(size_t)s].batch = -1;
    cv_work.notify_all();
  }

  ~Loader() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv_work.notify_all();
    cv_ready.notify_all();
    for (auto& t : workers) t.join();
  }
};

}  // namespace

#define MLR_EXPORT extern "C" __attribute__((visibility("default")))

MLR_EXPORT void* mlr_open(const char* path) {
  auto* rf = new RecordFile();
  rf->fd = open(path, O_RDONLY);
  struct stat st{};
  if (rf->fd < 0 || fstat(rf->fd, &st) != 0 || (size_t)st.st_size < sizeof(Header)) {
    if (rf->fd >= 0) close(rf->fd);
    delete rf;
    return nullptr;
  }
  rf->size = (size_t)st.st_size;
  void* m = mmap(nullptr, rf->size, PROT_READ, MAP_SHARED, rf->fd, 0);
  if (m == MAP_FAILED) { close(rf->fd); delete rf; return nullptr; }
  rf->map = (const uint8_t*)m;
  std::memcpy(&rf->h, rf->map, sizeof(Header));
  const uint64_t need = sizeof(Header) + rf->h.count * rf->h.record_bytes;
  if (std::memcmp(rf->h.magic, MAGIC, 8) != 0 || rf->h.label_bytes != 4 ||
      rf->h.record_bytes != (uint64_t)rf->h.H * rf->h.W * rf->h.C + 4 || need > rf->size || rf->h.count == 0) {
    munmap(m, rf->size);
    close(rf->fd);
    delete rf;
    return nullptr;
  }
  madvise(m, rf->size, MADV_RANDOM);
  return rf;
}

// shape[0..3] = count, H, W, C
MLR_EXPORT void mlr_shape(void* h, uint64_t* shape) {
  const auto* rf = (const RecordFile*)h;
  shape[0] = rf->h.count; shape[1] = rf->h.H; shape[2] = rf->h.W; shape[3] = rf->h.C;
}

MLR_EXPORT void mlr_close(void* h) {
  auto* rf = (RecordFile*)h;
  if (!rf) return;
  munmap((void*)rf->map, rf->size);
  close(rf->fd);
  delete rf;
}

// train != 0: RandomResizedCrop(scale [smin, smax], ratio [rmin, rmax]) + flip; else centre crop
MLR_EXPORT void* mlr_loader_create(void* file, int batch, int out_h, int out_w, int train, double smin, double smax,
                                   double rmin, double rmax, uint64_t seed, int rank, int world, int shuffle,
                                   int drop_last, int threads, int chunk) {
  if (!file || batch <= 0 || world <= 0 || rank < 0 || rank >= world || threads <= 0) return nullptr;
  auto* L = new Loader();
  L->rf = (const RecordFile*)file;
  L->batch = batch; L->out_h = out_h; L->out_w = out_w; L->train = train;
  L->smin = smin; L->smax = smax; L->rmin = rmin; L->rmax = rmax;
  L->seed = seed; L->rank = rank; L->world = world; L->shuffle = shuffle; L->drop_last = drop_last;
  L->chunk = chunk > 0 ? chunk : 16;
  for (int i = 0; i < threads; ++i) L->workers.emplace_back([L] { L->worker(); });
  return L;
}

// register ring slot `i` (call for every slot before the first epoch)
MLR_EXPORT int mlr_loader_set_slot(void* h, int i, uint8_t* img, int64_t* lab, int32_t* par) {
  auto* L = (Loader*)h;
  std::lock_guard<std::mutex> lk(L->mu);
  if (L->started || i < 0) return -1;
  if ((int)L->slots.size() <= i) L->slots.resize((size_t)i + 1);
  L->slots[(size_t)i].img = img;
  L->slots[(size_t)i].lab = lab;
  L->slots[(size_t)i].par = par;
  return 0;
}

// (re)start at `epoch`; returns the number of batches this rank yields in it
MLR_EXPORT int64_t mlr_loader_start_epoch(void* h, uint64_t epoch) {
  auto* L = (Loader*)h;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    if (L->slots.empty()) return -1;
    for (auto& s : L->slots)
      if (!s.img || !s.lab || !s.par) return -1;
  }
  L->start_epoch(epoch);
  return L->nbatches;
}

MLR_EXPORT int mlr_loader_next(void* h, int64_t* batch_index) { return ((Loader*)h)->next(batch_index); }
MLR_EXPORT void mlr_loader_release(void* h, int slot) { ((Loader*)h)->release(slot); }
MLR_EXPORT void mlr_loader_destroy(void* h) { delete (Loader*)h; }
