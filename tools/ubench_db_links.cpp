// The identifier job's DB writes alone (host only, no GPU, no files): what
// the step's "objects_links" phase costs in SqliteLibrary's bulk-identify
// mode, and in which order the rows are best written.
//
//   g++ -O2 -std=c++17 -Iinclude tools/ubench_db_links.cpp -Lspacedrive_amd -lsdcore -lsdcas \
//       -Wl,-rpath,$PWD/spacedrive_amd -Wl,-rpath-link,/opt/rocm/lib -o tools/ubench_db_links
//   tools/ubench_db_links [rows=100000] [batch=10000] [dup=0.15] [order=job|asc|many]
//
// A file database of `rows` file_path rows (C2-like: 100 directories), then
// the job's writes batch by batch: the batch's new Objects (create_objects)
// and one combined write per row (set_cas_id_and_connect), in the job's
// order (each created Object's first row, then the linked rows), in
// ascending row id, or in the job's order through set_cas_ids_and_connect
// (64 rows per UPDATE ... FROM (VALUES ...)). Prints the writes' seconds and the index rebuild's.
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sdcore.hpp"

using namespace sdcore;

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

int main(int argc, char** argv) {
  const size_t rows = argc > 1 ? strtoull(argv[1], nullptr, 10) : 100000;
  const size_t batch = argc > 2 ? strtoull(argv[2], nullptr, 10) : 10000;
  const double dup = argc > 3 ? atof(argv[3]) : 0.15;
  const bool asc = argc > 4 && !strcmp(argv[4], "asc");
  const bool many = argc > 4 && !strcmp(argv[4], "many");
  char tmpl[] = "/tmp/ubench_db_XXXXXX";
  if (!mkdtemp(tmpl)) return 1;
  const std::string path = std::string(tmpl) + "/lib.db";
  auto db = SqliteLibrary::open(path);
  std::vector<FilePathRow> fp(rows);
  for (size_t i = 0; i < rows; ++i) {
    fp[i].location_id = 1;
    fp[i].materialized_path = "/d" + std::to_string(i / 1000) + "/";
    fp[i].name = "f" + std::to_string(i);
    fp[i].extension = "bin";
    fp[i].size_in_bytes = 1 + mix(i) % 102400;
    fp[i].date_created = 1700000000 + (int64_t)i;
    fp[i].inode = 1000 + i;
  }
  db->add_file_paths(fp);
  // content per row: 15 % copies of an earlier row's content
  std::vector<uint64_t> content(rows);
  for (size_t i = 0; i < rows; ++i)
    content[i] = (i > 0 && (double)(mix(i ^ 0xABCD) % 10000) < dup * 10000) ? content[mix(i) % i] : i;
  auto cas_of = [](uint64_t c) {
    char b[17];
    snprintf(b, sizeof b, "%016llx", (unsigned long long)mix(c * 7 + 1));
    return std::string(b);
  };
  if (!db->begin_bulk_identify(rows)) {
    fprintf(stderr, "no bulk identify\n");
    return 1;
  }
  std::vector<int32_t> first_obj(rows, 0);  // content -> its Object
  double t_obj = 0, t_rows = 0;
  const double t0 = now();
  for (size_t b0 = 0; b0 < rows; b0 += batch) {
    const size_t b1 = std::min(rows, b0 + batch);
    db->begin_batch();
    double t = now();
    std::vector<size_t> creates;
    for (size_t i = b0; i < b1; ++i)
      if (content[i] == i) creates.push_back(i);
    std::vector<std::pair<ObjectKind, int64_t>> kd;
    for (size_t i : creates) kd.emplace_back(0, fp[i].date_created);
    const auto oids = db->create_objects(kd);
    for (size_t k = 0; k < creates.size(); ++k) first_obj[creates[k]] = oids[k];
    t_obj += now() - t;
    t = now();
    if (many) {
      std::vector<Library::CasLink> w;
      for (size_t i : creates) w.push_back({fp[i].id, cas_of(content[i]), first_obj[i]});
      for (size_t i = b0; i < b1; ++i)
        if (content[i] != i) w.push_back({fp[i].id, cas_of(content[i]), first_obj[content[i]]});
      db->set_cas_ids_and_connect(w);
    } else if (asc) {
      for (size_t i = b0; i < b1; ++i) db->set_cas_id_and_connect(fp[i].id, cas_of(content[i]), first_obj[content[i]]);
    } else {
      for (size_t i : creates) db->set_cas_id_and_connect(fp[i].id, cas_of(content[i]), first_obj[i]);
      for (size_t i = b0; i < b1; ++i)
        if (content[i] != i) db->set_cas_id_and_connect(fp[i].id, cas_of(content[i]), first_obj[content[i]]);
    }
    t_rows += now() - t;
    db->end_batch();
  }
  const double t_writes = now() - t0;
  const double t1 = now();
  db->end_bulk_identify();
  const double t_index = now() - t1;
  printf("{\"rows\": %zu, \"batch\": %zu, \"order\": \"%s\", \"writes_s\": %.4f, \"objects_s\": %.4f, "
         "\"row_writes_s\": %.4f, \"commit_s\": %.4f, \"index_s\": %.4f, \"rows_per_s\": %.0f}\n",
         rows, batch, many ? "many" : asc ? "asc" : "job", t_writes, t_obj, t_rows, t_writes - t_obj - t_rows, t_index,
         rows / (t_writes + t_index));
  unlink(path.c_str());
  unlink((path + "-wal").c_str());
  unlink((path + "-shm").c_str());
  rmdir(tmpl);
  return 0;
}
