// unipeak_amd/host/gzio.hpp -- the reference's stream filters by file-name
// suffix (misc/filterstream.cpp:30-50, 86-104; GZIP_SUFFIX / BZIP2_SUFFIX,
// misc/defaults.hpp:26-27): a name ending in ".gz" is read through a gzip
// decompressor and written through a gzip compressor (zlib, default level,
// like boost::iostreams' gzip filters).  ".bz2" would take bzip2 filters;
// libbz2's headers are not in this image, so such a name is refused with an
// "error:" line and exit 1 on both ends instead of being read or written as
// plain bytes.
#pragma once

#include <cstdio>
#include <string>

namespace unipeak {

bool is_gz(const std::string &fname);
bool is_bz2(const std::string &fname);

// fopen(fname, "rb") through the suffix's filter (".bz2": fatal).  nullptr
// when the file cannot be opened.
FILE *open_input(const std::string &fname);

// fopen(fname, "wb") through the suffix's filter (".bz2": fatal); fclose()
// finishes the gzip stream.  nullptr when the file cannot be created.
FILE *open_output(const std::string &fname);

// the whole decompressed content of a ".gz" file into out; false when the
// file cannot be opened; a corrupt stream is fatal
bool inflate_file(const std::string &fname, std::string &out);

}  // namespace unipeak
