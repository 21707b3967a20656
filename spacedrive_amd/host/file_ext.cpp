// ObjectKind of a file from its path: sd_file_ext's
// Extension::resolve_conflicting(path, always_check_magic_bytes = false)
// (crates/file-ext/src/magic.rs:176-235), as FileMetadata::new calls it
// (core/src/object/file_identifier/mod.rs:72-76), mapped to ObjectKind
// (crates/file-ext/src/kind.rs:4-59; extension_enum's From impl,
// magic.rs:82-88).
//
// Per category the accepted extension strings are the serde snake_case names
// of the category enum's variants (extensions.rs:32-363; every variant name is
// one capitalised word, so the name is its lowercase, plus the two renames
// "3gp" and "7z"). Extension::from_str lowercases the extension and collects
// the categories that accept it, in the Extension enum's order
// (extensions.rs:11-29): one match is the kind; two ("ts", "mts": Video and
// Code) are resolved by the video magic bytes; the file must open.

#include "sdcore.hpp"

#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

namespace sdcore {

namespace {

struct Category {
  ObjectKind kind;
  const char* names;  // space-separated, each with a leading and trailing space
};

// the Extension enum's categories in declaration order (extensions.rs:11-29)
const Category kCategories[] = {
    {ObjectKindDocument,
     " pdf key pages numbers doc docx xls xlsx ppt pptx odt ods odp ics hwp "},
    {ObjectKindVideo,
     " avi avifs qt mov swf mjpeg ts mts mpeg mxf m2v mpg mpe m2ts flv wm 3gp m4v wmv asf mp4 webm mkv vob ogv wtv "
     "hevc f4v "},
    {ObjectKindImage,
     " jpg jpeg png apng gif bmp tiff webp svg ico heic heics heif heifs hif avif avci avcs raw akw dng cr2 dcr nwr "
     "nef arw rw2 "},
    {ObjectKindAudio,
     " mp3 mp2 m4a wav aiff aif flac ogg oga opus wma amr aac wv voc tta loas caf aptx adts ast "},
    {ObjectKindArchive, " zip rar tar gz bz2 7z xz "},
    {ObjectKindExecutable, " exe app apk deb dmg pkg rpm msi jar bat "},
    {ObjectKindText, " txt rtf md markdown "},
    {ObjectKindEncrypted, " bytes container block "},
    {ObjectKindKey, " pgp pub pem p12 p8 keychain "},
    {ObjectKindFont, " ttf otf woff woff2 "},
    {ObjectKindMesh, " fbx obj "},
    {ObjectKindCode,
     " scpt scptd applescript sh zsh fish bash c cpp h hpp rb js mjs jsx html css sass scss less cr cs csx d dart "
     "dockerfile go hs java kt kts lua make nim nims m mm ml mli mll mly pl php php1 php2 php3 php4 php5 php6 phps "
     "phpt phtml ps1 psd1 psm1 py qml r rs sol sql swift ts tsx vala zig vue scala mdx astro mts "},
    {ObjectKindDatabase, " sqlite db "},
    {ObjectKindBook, " azw azw3 epub mobi "},
    {ObjectKindConfig, " ini json yaml yml toml xml mathml rss csv cfg compose tsconfig "},
};

// str::to_lowercase for the strings that can equal a name: ASCII letters
// fold, the Kelvin sign U+212A folds to 'k'; any other non-ASCII character
// keeps the result from matching (no name contains one) -> nullopt. Invalid
// UTF-8 cannot come through OsStr::to_str either (magic.rs:180).
std::optional<std::string> lowercase_for_match(const std::string& s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      out.push_back((char)(c >= 'A' && c <= 'Z' ? c + 32 : c));
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x84 && (unsigned char)s[i + 2] == 0xAA) {
      out.push_back('k');
      i += 2;
    } else {
      return std::nullopt;
    }
  }
  return out;
}

bool valid_utf8(const std::string& s) {
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (!n || i + n > s.size()) return false;
    for (size_t k = 1; k < n; ++k)
      if (((unsigned char)s[i + k] >> 6) != 2) return false;
    if (n == 2 && c < 0xC2) return false;  // overlong
    if (n == 3) {
      const unsigned char c1 = (unsigned char)s[i + 1];
      if ((c == 0xE0 && c1 < 0xA0) || (c == 0xED && c1 >= 0xA0)) return false;  // overlong / surrogate
    }
    if (n == 4) {
      const unsigned char c1 = (unsigned char)s[i + 1];
      if ((c == 0xF0 && c1 < 0x90) || c > 0xF4 || (c == 0xF4 && c1 >= 0x90)) return false;
    }
    i += n;
  }
  return true;
}

// Path::extension of a whole path: the last component's text after its last
// dot (std's rsplit_file_at_dot); trailing separators and "." components are
// not components; a last component ".." (or none) has no extension
std::optional<std::string> path_extension(const std::string& path) {
  std::string p = path;
  for (;;) {
    while (p.size() > 1 && p.back() == '/') p.pop_back();
    if (p.size() >= 2 && p.compare(p.size() - 2, 2, "/.") == 0) {
      p.resize(p.size() - 2);
      if (p.empty()) p = "/";
      continue;
    }
    break;
  }
  if (p.empty() || p == "/" || p == ".") return std::nullopt;
  const size_t slash = p.rfind('/');
  const std::string name = slash == std::string::npos ? p : p.substr(slash + 1);
  if (name.empty() || name == "..") return std::nullopt;
  return file_stem_and_extension(name).second;
}

// verify_magic_bytes (magic.rs:160-173): for each (offset, length) of the
// variant, read_exact that window (a short read ends the check: None) and
// match it against every byte pattern of the variant
bool read_exact_at(int fd, uint8_t* buf, size_t n, off_t off) {
  size_t got = 0;
  while (got < n) {
    const ssize_t r = ::pread(fd, buf + got, n - got, off + (off_t)got);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    got += (size_t)r;
  }
  return true;
}

// VideoExtension::Ts = [0x47] (extensions.rs:40): one window (0, 1)
bool video_ts_magic(int fd) {
  uint8_t b[1];
  return read_exact_at(fd, b, 1, 0) && b[0] == 0x47;
}

// VideoExtension::Mts = [0x47] | [_, _, _, 0x47] (extensions.rs:41): windows
// (0, 1) then (0, 4); each window is matched against both patterns
bool video_mts_magic(int fd) {
  uint8_t b[4];
  if (!read_exact_at(fd, b, 1, 0)) return false;
  if (b[0] == 0x47) return true;
  if (!read_exact_at(fd, b, 4, 0)) return false;
  return b[0] == 0x47 || b[3] == 0x47;
}

}  // namespace

std::vector<ObjectKind> extension_kinds(const std::string& ext) {
  std::vector<ObjectKind> out;
  auto low = lowercase_for_match(ext);
  if (!low || low->empty() || low->find(' ') != std::string::npos) return out;
  const std::string needle = " " + *low + " ";
  for (const auto& c : kCategories)
    if (std::strstr(c.names, needle.c_str())) out.push_back(c.kind);
  return out;
}

std::optional<ObjectKind> resolve_conflicting_kind(const std::string& path) {
  const auto ext = path_extension(path);
  if (!ext || !valid_utf8(*ext)) return std::nullopt;  // magic.rs:180-182
  const auto kinds = extension_kinds(*ext);           // magic.rs:184-186
  if (kinds.empty()) return std::nullopt;
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);  // magic.rs:188-190
  if (fd < 0) return std::nullopt;
  std::optional<ObjectKind> kind;
  if (kinds.size() == 1) {
    kind = kinds[0];  // Known: no magic check unless forced (magic.rs:195-215)
  } else {
    // Conflicts (magic.rs:217-233), matched on the extension as written
    bool video = false;
    for (ObjectKind k : kinds) video |= k == ObjectKindVideo;
    if (*ext == "ts" && video) kind = video_ts_magic(fd) ? ObjectKindVideo : ObjectKindCode;
    else if (*ext == "mts" && video) kind = video_mts_magic(fd) ? ObjectKindVideo : ObjectKindCode;
  }
  ::close(fd);
  return kind;
}

ObjectKind object_kind_of(const std::string& path) {
  return resolve_conflicting_kind(path).value_or(ObjectKindUnknown);  // mod.rs:73-76
}

}  // namespace sdcore
