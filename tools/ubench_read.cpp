// ubench_read.cpp — host read rate of many small files (measurement tool):
// the cas_id whole-file read pattern (cas.rs:27-29) through (a) open + pread
// + close per file on T threads, (b) io_uring on T threads, each ring keeping
// `depth` files in flight as linked OPENAT(direct) -> READ(fixed) ->
// CLOSE(direct) chains. Prints files/s and GB/s per mode.
//
//   ubench_read DIR NFILES THREADS DEPTH [reps]
// (DIR holds files 0000000..NFILES-1, as tools/e2e_bench.py writes them)
#include <fcntl.h>
#include <linux/io_uring.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static int sys_setup(unsigned entries, io_uring_params* p) { return (int)syscall(__NR_io_uring_setup, entries, p); }
static int sys_enter(int fd, unsigned to_submit, unsigned min_complete, unsigned flags) {
  return (int)syscall(__NR_io_uring_enter, fd, to_submit, min_complete, flags, nullptr, 0);
}
static int sys_register(int fd, unsigned op, const void* arg, unsigned nr) {
  return (int)syscall(__NR_io_uring_register, fd, op, arg, nr);
}

struct Ring {
  int fd = -1;
  unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
  io_uring_sqe* sqes;
  io_uring_cqe* cqes;
  unsigned sq_entries;
  unsigned local_tail;
  bool init(unsigned entries) {
    io_uring_params p;
    memset(&p, 0, sizeof p);
    fd = sys_setup(entries, &p);
    if (fd < 0) return false;
    sq_entries = p.sq_entries;
    size_t sq_sz = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    size_t cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    char* sq = (char*)mmap(nullptr, sq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQ_RING);
    char* cq = (char*)mmap(nullptr, cq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_CQ_RING);
    sqes = (io_uring_sqe*)mmap(nullptr, p.sq_entries * sizeof(io_uring_sqe), PROT_READ | PROT_WRITE,
                               MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQES);
    if (sq == MAP_FAILED || cq == MAP_FAILED || sqes == MAP_FAILED) return false;
    sq_head = (unsigned*)(sq + p.sq_off.head);
    sq_tail = (unsigned*)(sq + p.sq_off.tail);
    sq_mask = (unsigned*)(sq + p.sq_off.ring_mask);
    sq_array = (unsigned*)(sq + p.sq_off.array);
    cq_head = (unsigned*)(cq + p.cq_off.head);
    cq_tail = (unsigned*)(cq + p.cq_off.tail);
    cq_mask = (unsigned*)(cq + p.cq_off.ring_mask);
    cqes = (io_uring_cqe*)(cq + p.cq_off.cqes);
    local_tail = *sq_tail;
    return true;
  }
  io_uring_sqe* get() {
    unsigned head = __atomic_load_n(sq_head, __ATOMIC_ACQUIRE);
    if (local_tail - head >= sq_entries) return nullptr;
    unsigned idx = local_tail & *sq_mask;
    sq_array[idx] = idx;
    io_uring_sqe* s = &sqes[idx];
    memset(s, 0, sizeof *s);
    ++local_tail;
    return s;
  }
  unsigned flush() {
    unsigned n = local_tail - *sq_tail;
    __atomic_store_n(sq_tail, local_tail, __ATOMIC_RELEASE);
    return n;
  }
};

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s DIR NFILES THREADS DEPTH [reps]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int n = atoi(argv[2]), T = atoi(argv[3]), D = atoi(argv[4]), reps = argc > 5 ? atoi(argv[5]) : 3;
  std::vector<std::string> paths(n);
  std::vector<uint64_t> sizes(n);
  uint64_t total = 0;
  for (int i = 0; i < n; ++i) {
    char b[32];
    snprintf(b, sizeof b, "/%07d", i);
    paths[i] = dir + b;
    struct stat sb;
    if (stat(paths[i].c_str(), &sb)) {
      perror(paths[i].c_str());
      return 1;
    }
    sizes[i] = (uint64_t)sb.st_size;
    total += sizes[i];
  }
  // UB_NOATIME=1: open with O_NOATIME (no access-time update on read; the
  // caller must own the files)
  const int extra_flags = getenv("UB_NOATIME") ? O_NOATIME : 0;
  // (a) open + pread + close
  for (int r = 0; r < reps; ++r) {
    std::atomic<uint64_t> got{0};
    double t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        std::vector<char> buf(1 << 20);
        uint64_t g = 0;
        for (int i = t; i < n; i += T) {
          int fd = open(paths[i].c_str(), O_RDONLY | O_CLOEXEC | extra_flags);
          if (fd < 0) continue;
          ssize_t k = pread(fd, buf.data(), sizes[i] + 1, 0);
          if (k > 0) g += (uint64_t)k;
          close(fd);
        }
        got += g;
      });
    for (auto& x : th) x.join();
    double dt = now() - t0;
    printf("pread  T=%d: %.0f files/s %.2f GB/s (%s)\n", T, n / dt, total / dt / 1e9,
           got.load() == total ? "ok" : "SHORT");
  }
  // (b) io_uring: per ring `D` files in flight, fixed-file slots
  for (int r = 0; r < reps; ++r) {
    std::atomic<uint64_t> got{0};
    std::atomic<int> fail{0};
    double t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        Ring ring;
        if (!ring.init(4 * D)) {
          fail = 1;
          return;
        }
        std::vector<int> fds(D, -1);
        if (sys_register(ring.fd, IORING_REGISTER_FILES, fds.data(), D) < 0) {
          fail = 2;
          return;
        }
        std::vector<char> buf((size_t)D << 17);  // 128 KiB per slot (C2 files <= 100 KiB)
        std::vector<int> free_slots;
        for (int s = D - 1; s >= 0; --s) free_slots.push_back(s);
        int next = t, inflight = 0, errs = 0;
        uint64_t g = 0;
        while (next < n || inflight) {
          while (next < n && !free_slots.empty()) {
            int s = free_slots.back();
            free_slots.pop_back();
            io_uring_sqe* o = ring.get();
            o->opcode = IORING_OP_OPENAT;
            o->fd = AT_FDCWD;
            o->addr = (uint64_t)paths[next].c_str();
            o->open_flags = O_RDONLY;  // O_CLOEXEC is invalid for a direct descriptor
            o->file_index = s + 1;
            o->flags = IOSQE_IO_LINK;
            o->user_data = ((uint64_t)s << 32) | 0;
            io_uring_sqe* rd = ring.get();
            rd->opcode = IORING_OP_READ;
            rd->fd = s;
            rd->flags = IOSQE_FIXED_FILE | IOSQE_IO_LINK;
            rd->addr = (uint64_t)(buf.data() + ((size_t)s << 17));
            rd->len = (unsigned)(sizes[next] + 1);
            rd->off = 0;
            rd->user_data = ((uint64_t)s << 32) | 1;
            io_uring_sqe* c = ring.get();
            c->opcode = IORING_OP_CLOSE;
            c->file_index = s + 1;
            c->user_data = ((uint64_t)s << 32) | 2;
            ++inflight;
            next += T;
          }
          unsigned sub = ring.flush();
          sys_enter(ring.fd, sub, 1, IORING_ENTER_GETEVENTS);
          unsigned head = *ring.cq_head, tail = __atomic_load_n(ring.cq_tail, __ATOMIC_ACQUIRE);
          for (; head != tail; ++head) {
            io_uring_cqe* e = &ring.cqes[head & *ring.cq_mask];
            const int s = (int)(e->user_data >> 32), kind = (int)(e->user_data & 3);
            if (kind == 1 && e->res > 0) g += (uint64_t)e->res;
            if (e->res < 0 && kind != 2 && errs < 3) {
              ++errs;
              fprintf(stderr, "cqe kind %d res %d (%s)\n", kind, e->res, strerror(-e->res));
            }
            if (kind == 2) {
              free_slots.push_back(s);
              --inflight;
            }
          }
          __atomic_store_n(ring.cq_head, head, __ATOMIC_RELEASE);
        }
        got += g;
        close(ring.fd);
      });
    for (auto& x : th) x.join();
    double dt = now() - t0;
    if (fail) {
      printf("uring  T=%d D=%d: setup failed (%d)\n", T, D, fail.load());
      break;
    }
    printf("uring  T=%d D=%d: %.0f files/s %.2f GB/s (%s)\n", T, D, n / dt, total / dt / 1e9,
           got.load() == total ? "ok" : "SHORT");
  }
  return 0;
}
