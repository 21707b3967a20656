// sqlite3_min.h — the part of SQLite's public C API that SqliteLibrary uses.
// The image ships the library (libsqlite3.so.0, 3.37) without its
// development header; these declarations follow the documented, stable
// signatures of the SQLite C interface.
#pragma once
#include <stdint.h>

extern "C" {
struct sqlite3;
struct sqlite3_stmt;
typedef void (*sqlite3_destructor_type)(void*);

int sqlite3_open_v2(const char* filename, sqlite3** db, int flags, const char* vfs);
int sqlite3_close(sqlite3* db);
int sqlite3_exec(sqlite3* db, const char* sql, int (*cb)(void*, int, char**, char**), void* arg, char** errmsg);
void sqlite3_free(void* p);
const char* sqlite3_errmsg(sqlite3* db);
int sqlite3_prepare_v2(sqlite3* db, const char* sql, int nbyte, sqlite3_stmt** stmt, const char** tail);
int sqlite3_bind_int64(sqlite3_stmt* s, int i, int64_t v);
int sqlite3_bind_text(sqlite3_stmt* s, int i, const char* v, int n, sqlite3_destructor_type d);
int sqlite3_bind_blob(sqlite3_stmt* s, int i, const void* v, int n, sqlite3_destructor_type d);
int sqlite3_bind_null(sqlite3_stmt* s, int i);
int sqlite3_step(sqlite3_stmt* s);
int sqlite3_reset(sqlite3_stmt* s);
int sqlite3_clear_bindings(sqlite3_stmt* s);
int sqlite3_finalize(sqlite3_stmt* s);
int sqlite3_column_type(sqlite3_stmt* s, int i);
int64_t sqlite3_column_int64(sqlite3_stmt* s, int i);
const unsigned char* sqlite3_column_text(sqlite3_stmt* s, int i);
const void* sqlite3_column_blob(sqlite3_stmt* s, int i);
int sqlite3_column_bytes(sqlite3_stmt* s, int i);
int64_t sqlite3_last_insert_rowid(sqlite3* db);
int sqlite3_changes(sqlite3* db);
int sqlite3_busy_timeout(sqlite3* db, int ms);
}

constexpr int SQLITE_OK = 0;
constexpr int SQLITE_ROW = 100;
constexpr int SQLITE_DONE = 101;
constexpr int SQLITE_NULL = 5;
constexpr int SQLITE_OPEN_READONLY = 0x00000001;
constexpr int SQLITE_OPEN_READWRITE = 0x00000002;
constexpr int SQLITE_OPEN_CREATE = 0x00000004;
constexpr int SQLITE_OPEN_NOMUTEX = 0x00008000;
#define SQLITE_TRANSIENT ((sqlite3_destructor_type)-1)
