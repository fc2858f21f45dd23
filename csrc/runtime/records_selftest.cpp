// Self-test of the record loader (records.cpp), built with ThreadSanitizer and with
// AddressSanitizer + UBSan by mlcomp_amd.build.build_runtime_selftest (SURVEY §5.2 race
// detection for the native runtime).  It writes a record file, then drives the C API
// from one consumer thread the way the python RecordLoader does: several epochs, world
// sizes 1 and 3, thread counts 1..8, slow consumers, epochs abandoned half way.  Checks:
// every epoch of a rank yields each of its samples exactly once (no drop_last, count a
// multiple of world*batch), the sharded ranks partition the file, labels match the
// records, crop boxes lie inside the image, and two runs with different thread counts
// give the same stream.  Exit status 0 = pass.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* mlr_open(const char*);
void mlr_close(void*);
void mlr_shape(void*, uint64_t*);
void* mlr_loader_create(void*, int, int, int, int, double, double, double, double, uint64_t, int, int, int, int,
                        int, int);
int mlr_loader_set_slot(void*, int, uint8_t*, int64_t*, int32_t*);
int64_t mlr_loader_start_epoch(void*, uint64_t);
int mlr_loader_next(void*, int64_t*);
void mlr_loader_release(void*, int);
void mlr_loader_destroy(void*);
}

namespace {

constexpr int H = 12, W = 10, C = 3, N = 240;

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

void write_file(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "wb");
  CHECK(f);
  struct {
    char magic[8];
    uint32_t h, w, c, lb;
    uint64_t count, rb;
    uint8_t res[24];
  } hdr{};
  std::memcpy(hdr.magic, "MLREC001", 8);
  hdr.h = H; hdr.w = W; hdr.c = C; hdr.lb = 4; hdr.count = N; hdr.rb = H * W * C + 4;
  std::fwrite(&hdr, sizeof(hdr), 1, f);
  std::vector<uint8_t> img(H * W * C);
  for (int i = 0; i < N; ++i) {
    for (size_t j = 0; j < img.size(); ++j) img[j] = (uint8_t)(i * 7 + j);
    const int32_t lab = i;
    std::fwrite(img.data(), 1, img.size(), f);
    std::fwrite(&lab, 4, 1, f);
  }
  std::fclose(f);
}

// one rank's stream for `epochs` epochs: (label, box) per sample; abandon_at >= 0 stops
// each epoch after that many batches
std::vector<std::vector<int>> run(void* file, int batch, int world, int rank, int threads, int epochs,
                                  int abandon_at, int slow_us) {
  void* L = mlr_loader_create(file, batch, 8, 8, 1, 0.2, 1.0, 0.75, 1.333, 1234, rank, world, 1, 0, threads, 5);
  CHECK(L);
  const int depth = 3;
  std::vector<std::vector<uint8_t>> img(depth, std::vector<uint8_t>((size_t)batch * H * W * C));
  std::vector<std::vector<int64_t>> lab(depth, std::vector<int64_t>(batch));
  std::vector<std::vector<int32_t>> par(depth, std::vector<int32_t>((size_t)batch * 5));
  for (int i = 0; i < depth; ++i) CHECK(mlr_loader_set_slot(L, i, img[i].data(), lab[i].data(), par[i].data()) == 0);
  std::vector<std::vector<int>> out;
  for (int e = 0; e < epochs; ++e) {
    const int64_t nb = mlr_loader_start_epoch(L, (uint64_t)e);
    CHECK(nb == (N / world + batch - 1) / batch);
    std::vector<int> seen;
    for (int64_t b = 0; b < nb; ++b) {
      if (abandon_at >= 0 && b == abandon_at) break;
      int64_t bi = -1;
      const int s = mlr_loader_next(L, &bi);
      CHECK(s >= 0 && bi == b);
      for (int i = 0; i < batch; ++i) {
        const int l = (int)lab[s][i];
        CHECK(l >= 0 && l < N);
        CHECK(img[s][(size_t)i * H * W * C] == (uint8_t)(l * 7));   // pixels belong to that record
        const int32_t* p = &par[s][(size_t)i * 5];
        CHECK(p[2] > 0 && p[3] > 0 && p[0] >= 0 && p[1] >= 0 && p[0] + p[2] <= H && p[1] + p[3] <= W);
        CHECK(p[4] == 0 || p[4] == 1);
        seen.push_back(l);
        seen.push_back(p[0] * 1000000 + p[1] * 10000 + p[2] * 100 + p[3] * 2 + p[4]);
      }
      if (slow_us) std::this_thread::sleep_for(std::chrono::microseconds(slow_us));
      mlr_loader_release(L, s);
    }
    out.push_back(seen);
  }
  mlr_loader_destroy(L);
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string path = std::string(argc > 1 ? argv[1] : "/tmp") + "/selftest.mlrec";
  write_file(path);
  void* f = mlr_open(path.c_str());
  CHECK(f);
  uint64_t shp[4];
  mlr_shape(f, shp);
  CHECK(shp[0] == N && shp[1] == H && shp[2] == W && shp[3] == C);
  // determinism across thread counts and consumer speed
  const auto ref = run(f, 8, 1, 0, 1, 3, -1, 0);
  for (int th : {2, 5, 8}) CHECK(run(f, 8, 1, 0, th, 3, -1, th == 5 ? 200 : 0) == ref);
  // each epoch is a permutation; epochs differ
  for (const auto& ep : ref) {
    std::set<int> labs;
    for (size_t i = 0; i < ep.size(); i += 2) labs.insert(ep[i]);
    CHECK((int)labs.size() == N);
  }
  CHECK(ref[0] != ref[1]);
  // sharding: 3 ranks partition every epoch
  for (int e = 0; e < 2; ++e) {
    std::set<int> all;
    size_t total = 0;
    for (int r = 0; r < 3; ++r) {
      const auto s = run(f, 10, 3, r, 4, 2, -1, 0);
      for (size_t i = 0; i < s[(size_t)e].size(); i += 2) all.insert(s[(size_t)e][i]);
      total += s[(size_t)e].size() / 2;
    }
    CHECK((int)all.size() == N && (int)total == N);
  }
  // abandoned epochs (consumer stops early) restart cleanly
  for (int th : {1, 6}) {
    const auto a = run(f, 8, 1, 0, th, 4, 2, 0);
    for (size_t e = 0; e < a.size(); ++e) CHECK(a[e].size() == 2 * 2 * 8);
  }
  mlr_close(f);
  std::remove(path.c_str());
  std::printf("records selftest ok\n");
  return 0;
}
