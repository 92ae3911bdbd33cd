// _kwcore — native watch-event decoder for k8s-watcher-amd.
//
// Hot path of the watcher: one kube-apiserver watch line
// `{"type":"MODIFIED","object":{<Pod>}}` → the fields the filters need plus the
// clusterapi payload *core* (reference
// /root/reference/watcher/pod_watcher.py:159-202) as ready-to-send JSON bytes.
//
// The reference pays for this with json.loads + reflective V1Pod model
// construction inside the `kubernetes` library and then a Python dict build;
// here a single forward pass over the line records byte spans of the ~20
// fields that matter, skips everything else (managedFields, volumes, env, ...)
// with a structural scanner, and assembles the payload by copying raw JSON
// tokens. No Python object is created for the pod body.
//
// Semantics are pinned to the Python engine (models/payload.py::build_core),
// see tests/test_native_parity.py.

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <arpa/inet.h>
#include <fcntl.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <linux/futex.h>
#include <malloc.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/sendfile.h>
#include <sys/resource.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <sys/types.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <array>
#include <charconv>
#include <chrono>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace {

// ----------------------------------------------------------------------------- spans

struct Span {
    const char* p = nullptr;  // raw JSON token (strings include their quotes)
    size_t n = 0;
    bool present() const { return p != nullptr; }
    bool is_null() const { return p && n == 4 && std::memcmp(p, "null", 4) == 0; }
    bool is_string() const { return p && n >= 2 && p[0] == '"'; }
};

struct Condition { Span type, status, reason, message; };
struct CStatus { Span name, ready, restart_count, state; };
struct Container { Span name, image; };

struct PodSpans {
    bool meta_present = false;
    Span name, ns, uid, rv, labels, annotations, ctime, owners;
    Span pod_ip, host_ip, start_time, qos;  // watcher.payload_extra_fields
    bool spec_present = false;
    Span node_name;
    std::vector<Container> containers;
    bool status_present = false;
    Span phase;
    std::vector<Condition> conditions;
    std::vector<CStatus> cstatuses;
    bool deferred = false;             // parse_pod_light: spec/arrays not walked yet
    Span spec_raw, cond_raw, cstat_raw;
    void clear() {
        meta_present = spec_present = status_present = deferred = false;
        name = ns = uid = rv = labels = annotations = ctime = node_name = phase = Span();
        owners = pod_ip = host_ip = start_time = qos = Span();
        spec_raw = cond_raw = cstat_raw = Span();
        containers.clear();
        conditions.clear();
        cstatuses.clear();
    }
};

struct ParseError {
    const char* msg;
};

// ----------------------------------------------------------------------------- scanner

class Parser {
  public:
    Parser(const char* b, const char* e) : p_(b), end_(e) {}
    const char* p_;
    const char* end_;

    [[noreturn]] void fail(const char* m) { throw ParseError{m}; }

    inline void ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
    }
    inline char peek() {
        ws();
        if (p_ >= end_) fail("unexpected end of input");
        return *p_;
    }
    inline void expect(char c) {
        if (peek() != c) fail("unexpected character");
        ++p_;
    }

    // Returns pointer one past the closing quote of the string starting at p_ ('"').
    inline const char* string_end(const char* s) {
        ++s;  // opening quote
#if defined(__x86_64__)
        if (use_avx2) return string_end_avx2(s);
#endif
        while (s < end_) {
            char c = *s;
            if (c == '"') return s + 1;
            if (c == '\\') {
                s += 2;
                continue;
            }
            ++s;
        }
        fail("unterminated string");
    }

#if defined(__x86_64__)
    static bool use_avx2;
    static bool use_avx512;
    __attribute__((target("avx2,bmi,bmi2"))) const char* string_end_avx2(const char* s) {
        const __m256i q = _mm256_set1_epi8('"');
        const __m256i bs = _mm256_set1_epi8('\\');
        while (s + 32 <= end_) {
            __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s));
            uint32_t mq = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, q));
            uint32_t mb = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, bs));
            if (mb == 0) {
                if (mq) return s + __builtin_ctz(mq) + 1;
                s += 32;
                continue;
            }
            uint32_t first_b = __builtin_ctz(mb);
            if (mq && (uint32_t)__builtin_ctz(mq) < first_b) return s + __builtin_ctz(mq) + 1;
            s += first_b + 2;  // skip the escape pair, rescan from there
        }
        while (s < end_) {
            char c = *s;
            if (c == '"') return s + 1;
            if (c == '\\') {
                s += 2;
                continue;
            }
            ++s;
        }
        fail("unterminated string");
    }

    // Skip a balanced {...} or [...] starting at s (the opener), 64 bytes per
    // step: structural-character bitmasks from two AVX2 compares, escaped
    // quotes removed with the odd-backslash-run rule, string interiors masked
    // with a carry-less-multiply prefix XOR, and the bracket depth advanced
    // by popcounts; bits are only walked one by one in the block where the
    // depth can return to zero.
    static inline __attribute__((target("avx2"))) uint64_t mask64(__m256i lo, __m256i hi, __m256i c) {
        uint32_t a = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(lo, c));
        uint32_t b = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(hi, c));
        return (uint64_t)a | ((uint64_t)b << 32);
    }

    static inline uint64_t escaped_mask(uint64_t backslash, uint64_t& prev_escaped) {
        const uint64_t even = 0x5555555555555555ULL;
        backslash &= ~prev_escaped;
        uint64_t follows = (backslash << 1) | prev_escaped;
        uint64_t odd_starts = backslash & ~even & ~follows;
        uint64_t seq_even;
        prev_escaped = __builtin_add_overflow(odd_starts, backslash, &seq_even) ? 1 : 0;
        uint64_t invert = seq_even << 1;
        return (even ^ invert) & follows;
    }

    __attribute__((target("avx2,bmi,bmi2,pclmul,popcnt"))) const char* skip_container_blocks(const char* s) {
        uint64_t prev_escaped = 0, prev_in_string = 0;
        int64_t depth = 0;
        const char* p = s;
        alignas(32) char tail[64];
        const __m256i vq = _mm256_set1_epi8('"'), vb = _mm256_set1_epi8('\\');
        const __m256i vob = _mm256_set1_epi8('{'), vcb = _mm256_set1_epi8('}');
        const __m256i v20 = _mm256_set1_epi8(0x20);
        while (p < end_) {
            size_t avail = (size_t)(end_ - p);
            const char* blk = p;
            uint64_t valid = ~0ULL;
            if (avail < 64) {
                std::memset(tail, ' ', sizeof tail);
                std::memcpy(tail, p, avail);
                blk = tail;
                valid = (1ULL << avail) - 1;
            }
            __m256i lo = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk));
            __m256i hi = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + 32));
            uint64_t quotes = mask64(lo, hi, vq) & ~escaped_mask(mask64(lo, hi, vb), prev_escaped);
            uint64_t in_str = (uint64_t)_mm_cvtsi128_si64(
                _mm_clmulepi64_si128(_mm_set_epi64x(0, (long long)quotes), _mm_set1_epi8((char)0xFF), 0));
            in_str ^= prev_in_string;
            prev_in_string = (uint64_t)((int64_t)in_str >> 63);
            // '{'|0x20 == '['|0x20 == '{' and '}'|0x20 == ']'|0x20 == '}': one compare per bracket kind
            const __m256i lo20 = _mm256_or_si256(lo, v20), hi20 = _mm256_or_si256(hi, v20);
            uint64_t open = mask64(lo20, hi20, vob) & ~in_str & valid;
            uint64_t close = mask64(lo20, hi20, vcb) & ~in_str & valid;
            int64_t nclose = __builtin_popcountll(close);
            if (depth > nclose) {
                depth += __builtin_popcountll(open) - nclose;
            } else {
                uint64_t m = open | close;
                while (m) {
                    int i = __builtin_ctzll(m);
                    if ((open >> i) & 1) {
                        ++depth;
                    } else if (--depth == 0) {
                        return p + i + 1;
                    }
                    m &= m - 1;
                }
            }
            p += avail < 64 ? avail : 64;
        }
        fail("unterminated container");
    }

    // AVX-512BW form of the same block scanner (Zen 4/5 and recent Xeons run
    // 512-bit compares at full width): one load and four compares yield the
    // 64-bit quote/backslash/open/close masks directly in mask registers, the
    // escape pass is skipped for blocks with no backslash, and the final
    // partial block is a fault-suppressing masked load instead of a copy.
    __attribute__((target("avx512f,avx512bw,bmi,bmi2,pclmul,popcnt"))) const char* skip_container_512(
        const char* s) {
        uint64_t prev_escaped = 0, prev_in_string = 0;
        int64_t depth = 0;
        const char* p = s;
        const __m512i vq = _mm512_set1_epi8('"'), vb = _mm512_set1_epi8('\\');
        const __m512i vo = _mm512_set1_epi8('{'), vc = _mm512_set1_epi8('}'), v20 = _mm512_set1_epi8(0x20);
        while (p < end_) {
            size_t avail = (size_t)(end_ - p);
            uint64_t valid = ~0ULL;
            __m512i v;
            if (avail >= 64) {
                v = _mm512_loadu_si512(reinterpret_cast<const void*>(p));
            } else {
                valid = (1ULL << avail) - 1;
                v = _mm512_maskz_loadu_epi8(valid, p);
            }
            uint64_t quotes = _mm512_cmpeq_epi8_mask(v, vq);
            uint64_t bs = _mm512_cmpeq_epi8_mask(v, vb);
            if (bs | prev_escaped) quotes &= ~escaped_mask(bs, prev_escaped);
            uint64_t in_str = (uint64_t)_mm_cvtsi128_si64(
                _mm_clmulepi64_si128(_mm_set_epi64x(0, (long long)quotes), _mm_set1_epi8((char)0xFF), 0));
            in_str ^= prev_in_string;
            prev_in_string = (uint64_t)((int64_t)in_str >> 63);
            const __m512i f = _mm512_or_si512(v, v20);
            uint64_t open = _mm512_cmpeq_epi8_mask(f, vo) & ~in_str & valid;
            uint64_t close = _mm512_cmpeq_epi8_mask(f, vc) & ~in_str & valid;
            int64_t nclose = __builtin_popcountll(close);
            if (depth > nclose) {
                depth += __builtin_popcountll(open) - nclose;
            } else {
                uint64_t m = open | close;
                while (m) {
                    int i = __builtin_ctzll(m);
                    if ((open >> i) & 1) {
                        ++depth;
                    } else if (--depth == 0) {
                        return p + i + 1;
                    }
                    m &= m - 1;
                }
            }
            p += avail < 64 ? avail : 64;
        }
        fail("unterminated container");
    }

    __attribute__((target("avx2,bmi,bmi2"))) const char* skip_container_avx2(const char* s) {
        int depth = 0;
        const __m256i q = _mm256_set1_epi8('"');
        const __m256i ob = _mm256_set1_epi8('{');
        const __m256i cb = _mm256_set1_epi8('}');
        const __m256i os = _mm256_set1_epi8('[');
        const __m256i cs = _mm256_set1_epi8(']');
        while (s + 32 <= end_) {
            __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s));
            uint32_t m = (uint32_t)_mm256_movemask_epi8(
                _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi8(v, q), _mm256_cmpeq_epi8(v, ob)),
                                _mm256_or_si256(_mm256_cmpeq_epi8(v, cb),
                                                _mm256_or_si256(_mm256_cmpeq_epi8(v, os),
                                                                _mm256_cmpeq_epi8(v, cs)))));
            const char* next = s + 32;
            while (m) {
                uint32_t i = __builtin_ctz(m);
                const char* c = s + i;
                char ch = *c;
                if (ch == '"') {
                    const char* after = string_end_avx2(c + 1);
                    if (after > s + 32) {
                        next = after;
                        m = 0;
                        break;
                    }
                    // clear bits up to and including the closing quote
                    uint32_t upto = (uint32_t)(after - s);
                    m = upto >= 32 ? 0 : (m & ~((1u << upto) - 1u));
                    if (upto >= 32) {
                        next = after;
                        break;
                    }
                    continue;
                }
                if (ch == '{' || ch == '[') {
                    ++depth;
                } else {
                    if (--depth == 0) return c + 1;
                }
                m &= m - 1;
            }
            s = next;
        }
        return skip_container_scalar(s, depth);
    }
#endif

    const char* skip_container_scalar(const char* s, int depth) {
        while (s < end_) {
            char c = *s;
            if (c == '"') {
                s = string_end_scalar(s + 1);
                continue;
            }
            if (c == '{' || c == '[') {
                ++depth;
            } else if (c == '}' || c == ']') {
                if (--depth == 0) return s + 1;
            }
            ++s;
        }
        fail("unterminated container");
    }

    const char* string_end_scalar(const char* s) {
        while (s < end_) {
            char c = *s;
            if (c == '"') return s + 1;
            if (c == '\\') {
                s += 2;
                continue;
            }
            ++s;
        }
        fail("unterminated string");
    }

    // Skip any JSON value at p_ and return its raw span.
    Span value() {
        char c = peek();
        Span sp;
        sp.p = p_;
        if (c == '"') {
            p_ = string_end(p_);
        } else if (c == '{' || c == '[') {
#if defined(__x86_64__)
            p_ = use_avx512 ? skip_container_512(p_)
                 : use_avx2 ? skip_container_blocks(p_)
                            : skip_container_scalar(p_, 0);
#else
            p_ = skip_container_scalar(p_, 0);
#endif
        } else {
            while (p_ < end_) {
                char d = *p_;
                if (d == ',' || d == '}' || d == ']' || d == ' ' || d == '\n' || d == '\r' || d == '\t') break;
                ++p_;
            }
            if (p_ == sp.p) fail("empty value");
        }
        sp.n = (size_t)(p_ - sp.p);
        return sp;
    }

    // Read an object key (raw, without quotes; escapes left as-is — keys we
    // match never contain escapes) and consume the following ':'.
    inline void key(const char*& k, size_t& kn) {
        if (peek() != '"') fail("expected key");
        const char* s = p_ + 1;
        p_ = string_end(p_);
        k = s;
        kn = (size_t)(p_ - 1 - s);
        expect(':');
    }

    // Iterate an object: f(key, keylen) must consume the value.
    template <class F>
    void object(F&& f) {
        expect('{');
        if (peek() == '}') {
            ++p_;
            return;
        }
        while (true) {
            const char* k;
            size_t kn;
            key(k, kn);
            f(k, kn);
            char c = peek();
            ++p_;
            if (c == '}') return;
            if (c != ',') fail("expected , or }");
        }
    }

    template <class F>
    void array(F&& f) {
        expect('[');
        if (peek() == ']') {
            ++p_;
            return;
        }
        while (true) {
            f();
            char c = peek();
            ++p_;
            if (c == ']') return;
            if (c != ',') fail("expected , or ]");
        }
    }

    bool null_here() {
        if (peek() == 'n' && end_ - p_ >= 4 && std::memcmp(p_, "null", 4) == 0) {
            p_ += 4;
            return true;
        }
        return false;
    }
};

#if defined(__x86_64__)
bool Parser::use_avx2 = false;
bool Parser::use_avx512 = false;

bool simd_supported() {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi2") &&
           __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("popcnt");
}

bool avx512_supported() {
    __builtin_cpu_init();
    return simd_supported() && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
}
#endif

#define KEYIS(lit) (kn == sizeof(lit) - 1 && std::memcmp(k, lit, sizeof(lit) - 1) == 0)

void parse_metadata(Parser& P, PodSpans& S) {
    // a repeated "metadata" key replaces the first one whole (json.loads: the last key wins)
    S.meta_present = false;
    S.name = S.ns = S.uid = S.rv = S.labels = S.annotations = S.ctime = S.owners = Span();
    if (P.null_here()) return;
    S.meta_present = true;
    P.object([&](const char* k, size_t kn) {
        switch (kn) {
            case 3:
                if (KEYIS("uid")) { S.uid = P.value(); return; }
                break;
            case 4:
                if (KEYIS("name")) { S.name = P.value(); return; }
                break;
            case 6:
                if (KEYIS("labels")) { S.labels = P.value(); return; }
                break;
            case 9:
                if (KEYIS("namespace")) { S.ns = P.value(); return; }
                break;
            case 11:
                if (KEYIS("annotations")) { S.annotations = P.value(); return; }
                break;
            case 15:
                if (KEYIS("resourceVersion")) { S.rv = P.value(); return; }
                if (KEYIS("ownerReferences")) { S.owners = P.value(); return; }
                break;
            case 17:
                if (KEYIS("creationTimestamp")) { S.ctime = P.value(); return; }
                break;
        }
        P.value();
    });
}

// "metadata" present but not an object or null: as absent (the Python engine reads it as {})
void parse_metadata_absent(PodSpans& S) {
    S.meta_present = false;
    S.name = S.ns = S.uid = S.rv = S.labels = S.annotations = S.ctime = S.owners = Span();
}

void parse_containers(Parser& P, PodSpans& S) {
    S.containers.clear();  // a repeated key replaces the list (json.loads: the last key wins)
    if (P.null_here()) return;
    if (P.peek() != '[') { P.value(); return; }
    P.array([&]() {
        if (P.peek() != '{') { P.value(); return; }
        Container c;
        P.object([&](const char* k, size_t kn) {
            if (KEYIS("name")) c.name = P.value();
            else if (KEYIS("image")) c.image = P.value();
            else P.value();
        });
        S.containers.push_back(c);
    });
}

void parse_conditions(Parser& P, PodSpans& S) {
    S.conditions.clear();  // a repeated key replaces the list (json.loads: the last key wins)
    if (P.null_here()) return;
    if (P.peek() != '[') { P.value(); return; }
    P.array([&]() {
        if (P.peek() != '{') { P.value(); return; }
        Condition c;
        P.object([&](const char* k, size_t kn) {
            if (KEYIS("type")) c.type = P.value();
            else if (KEYIS("status")) c.status = P.value();
            else if (KEYIS("reason")) c.reason = P.value();
            else if (KEYIS("message")) c.message = P.value();
            else P.value();
        });
        S.conditions.push_back(c);
    });
}

void parse_cstatuses(Parser& P, PodSpans& S) {
    S.cstatuses.clear();  // a repeated key replaces the list (json.loads: the last key wins)
    if (P.null_here()) return;
    if (P.peek() != '[') { P.value(); return; }
    P.array([&]() {
        if (P.peek() != '{') { P.value(); return; }
        CStatus c;
        P.object([&](const char* k, size_t kn) {
            if (KEYIS("name")) c.name = P.value();
            else if (KEYIS("ready")) c.ready = P.value();
            else if (KEYIS("restartCount")) c.restart_count = P.value();
            else if (KEYIS("state")) c.state = P.value();
            else P.value();
        });
        S.cstatuses.push_back(c);
    });
}

void reset_spec(PodSpans& S) {
    S.spec_present = false;
    S.node_name = S.spec_raw = Span();
    S.containers.clear();
}

void reset_status(PodSpans& S) {
    S.status_present = false;
    S.phase = S.pod_ip = S.host_ip = S.start_time = S.qos = S.cond_raw = S.cstat_raw = Span();
    S.conditions.clear();
    S.cstatuses.clear();
}

void parse_spec(Parser& P, PodSpans& S) {
    if (P.null_here()) return;
    S.spec_present = true;
    P.object([&](const char* k, size_t kn) {
        if (KEYIS("nodeName")) S.node_name = P.value();
        else if (KEYIS("containers")) parse_containers(P, S);
        else P.value();
    });
}

// status scalars for watcher.payload_extra_fields (a few length-gated compares)
bool status_scalar(Parser& P, PodSpans& S, const char* k, size_t kn) {
    switch (kn) {
        case 5:
            if (KEYIS("podIP")) { S.pod_ip = P.value(); return true; }
            break;
        case 6:
            if (KEYIS("hostIP")) { S.host_ip = P.value(); return true; }
            break;
        case 8:
            if (KEYIS("qosClass")) { S.qos = P.value(); return true; }
            break;
        case 9:
            if (KEYIS("startTime")) { S.start_time = P.value(); return true; }
            break;
    }
    return false;
}

void parse_status(Parser& P, PodSpans& S) {
    if (P.null_here()) return;
    S.status_present = true;
    P.object([&](const char* k, size_t kn) {
        if (KEYIS("phase")) S.phase = P.value();
        else if (KEYIS("conditions")) parse_conditions(P, S);
        else if (KEYIS("containerStatuses")) parse_cstatuses(P, S);
        else if (!status_scalar(P, S, k, kn)) P.value();
    });
}

void parse_pod(Parser& P, PodSpans& S) {
    P.object([&](const char* k, size_t kn) {
        if (KEYIS("metadata")) {
            if (P.peek() == '{' || P.peek() == 'n') {
                parse_metadata(P, S);
            } else {
                P.value();
                parse_metadata_absent(S);
            }
        } else if (KEYIS("spec")) {
            reset_spec(S);
            if (P.peek() == '{' || P.peek() == 'n') parse_spec(P, S); else P.value();
        } else if (KEYIS("status")) {
            reset_status(S);
            if (P.peek() == '{' || P.peek() == 'n') parse_status(P, S); else P.value();
        } else {
            P.value();
        }
    });
}

// Filter-first variant for the fused pipeline: everything the filters and the
// cache need (metadata, status.phase) is extracted, while spec and the two
// status arrays are only bracket-skipped by the block scanner and their raw
// spans kept; materialize() walks them later for the events that actually get
// a payload. With the critical-events filter ~4 of 5 churn events never pay
// for the container/condition walk.
void parse_status_light(Parser& P, PodSpans& S) {
    if (P.null_here()) return;
    S.status_present = true;
    P.object([&](const char* k, size_t kn) {
        if (KEYIS("phase")) S.phase = P.value();
        else if (KEYIS("conditions")) S.cond_raw = P.value();
        else if (KEYIS("containerStatuses")) S.cstat_raw = P.value();
        else if (!status_scalar(P, S, k, kn)) P.value();
    });
}

void parse_pod_light(Parser& P, PodSpans& S) {
    S.deferred = true;
    P.object([&](const char* k, size_t kn) {
        if (KEYIS("metadata")) {
            if (P.peek() == '{' || P.peek() == 'n') {
                parse_metadata(P, S);
            } else {
                P.value();
                parse_metadata_absent(S);
            }
        } else if (KEYIS("spec")) {
            reset_spec(S);
            char c = P.peek();
            if (c == '{') {
                S.spec_present = true;
                S.spec_raw = P.value();
            } else if (!P.null_here()) {
                P.value();
            }
        } else if (KEYIS("status")) {
            reset_status(S);
            if (P.peek() == '{' || P.peek() == 'n') parse_status_light(P, S); else P.value();
        } else {
            P.value();
        }
    });
}

// Walk the sub-trees parse_pod_light deferred; throws ParseError like parse_pod.
void materialize(PodSpans& S) {
    if (!S.deferred) return;
    S.deferred = false;
    if (S.spec_raw.present()) {
        Parser Q(S.spec_raw.p, S.spec_raw.p + S.spec_raw.n);
        parse_spec(Q, S);
    }
    if (S.cond_raw.present()) {
        Parser Q(S.cond_raw.p, S.cond_raw.p + S.cond_raw.n);
        parse_conditions(Q, S);
    }
    if (S.cstat_raw.present()) {
        Parser Q(S.cstat_raw.p, S.cstat_raw.p + S.cstat_raw.n);
        parse_cstatuses(Q, S);
    }
}

// ----------------------------------------------------------------------------- output

inline void put(std::string& o, const char* s, size_t n) { o.append(s, n); }
inline void put(std::string& o, const char* lit) { o.append(lit); }
inline void raw_or_null(std::string& o, const Span& s) {
    if (s.present()) o.append(s.p, s.n); else o.append("null", 4);
}

// JSON "falsy" per Python truthiness after json.loads: null, {}, [], "", 0, false.
bool falsy_token(const Span& s) {
    if (!s.present()) return true;
    const char* p = s.p;
    size_t n = s.n;
    if (n == 4 && std::memcmp(p, "null", 4) == 0) return true;
    if (n == 5 && std::memcmp(p, "false", 5) == 0) return true;
    if (n == 2 && std::memcmp(p, "\"\"", 2) == 0) return true;
    if (p[0] == '{' || p[0] == '[') {
        for (size_t i = 1; i + 1 < n; ++i) {
            char c = p[i];
            if (!(c == ' ' || c == '\n' || c == '\r' || c == '\t')) return false;
        }
        return true;
    }
    if (p[0] == '0' || p[0] == '-') {
        for (size_t i = 0; i < n; ++i) {
            char c = p[i];
            if (c != '0' && c != '-' && c != '.' && c != 'e' && c != 'E' && c != '+') return false;
        }
        return true;
    }
    return false;
}

bool is_digit(char c) { return c >= '0' && c <= '9'; }

// models/timefmt.py::k8s_time_to_isoformat on the raw string token.
void creation_time(std::string& o, const Span& s) {
    if (!s.present() || s.is_null()) {
        o.append("null", 4);
        return;
    }
    if (!s.is_string()) {  // non-string: passed through unchanged
        o.append(s.p, s.n);
        return;
    }
    const char* p = s.p + 1;
    size_t n = s.n - 2;
    for (size_t i = 0; i < n; ++i)
        if (p[i] == '\\') {  // never produced by the API; keep verbatim
            o.append(s.p, s.n);
            return;
        }
    // YYYY-MM-DD[Tt ]HH:MM:SS(.frac)?(Z|z|[+-]HH:?MM)?
    auto digits = [&](size_t at, size_t cnt) {
        if (at + cnt > n) return false;
        for (size_t i = 0; i < cnt; ++i)
            if (!is_digit(p[at + i])) return false;
        return true;
    };
    bool ok = n >= 19 && digits(0, 4) && p[4] == '-' && digits(5, 2) && p[7] == '-' && digits(8, 2) &&
              (p[10] == 'T' || p[10] == 't' || p[10] == ' ') && digits(11, 2) && p[13] == ':' &&
              digits(14, 2) && p[16] == ':' && digits(17, 2);
    size_t i = 19;
    size_t fs = 0, fn = 0;
    if (ok && i < n && p[i] == '.') {
        fs = ++i;
        while (i < n && is_digit(p[i])) ++i;
        fn = i - fs;
        if (fn == 0) ok = false;
    }
    std::string tz;
    bool has_tz = false;
    if (ok && i < n) {
        if ((p[i] == 'Z' || p[i] == 'z') && i + 1 == n) {
            tz = "+00:00";
            has_tz = true;
        } else if ((p[i] == '+' || p[i] == '-') && (n - i == 6 || n - i == 5)) {
            if (n - i == 6 && digits(i + 1, 2) && p[i + 3] == ':' && digits(i + 4, 2)) {
                tz.assign(p + i, 6);
            } else if (n - i == 5 && digits(i + 1, 4)) {
                tz.assign(p + i, 3);
                tz.push_back(':');
                tz.append(p + i + 3, 2);
            } else {
                ok = false;
            }
            if (tz == "-00:00") tz = "+00:00";
            has_tz = true;
        } else {
            ok = false;
        }
    }
    if (!ok) {
        o.append(s.p, s.n);
        return;
    }
    o.push_back('"');
    o.append(p, 10);
    o.push_back('T');
    o.append(p + 11, 8);
    if (fn) {
        char micro[7];
        for (size_t k = 0; k < 6; ++k) micro[k] = k < fn ? p[fs + k] : '0';
        micro[6] = 0;
        bool nonzero = false;
        for (size_t k = 0; k < 6; ++k)
            if (micro[k] != '0') nonzero = true;
        if (nonzero) {
            o.push_back('.');
            o.append(micro, 6);
        }
    }
    if (has_tz) o.append(tz);
    o.push_back('"');
}

// extra: bit i = models/payload.py EXTRA_FIELDS[i]
// (pod_ip, host_ip, start_time, qos_class, resource_version, owner_references)
bool state_repr_json(std::string& o, const Span& state, const std::string& tz_utc);  // pyrepr.inc

// tz_utc non-null: watcher.state_format python_repr (pyrepr.inc); false when
// a state needs the Python formatter (the core is then incomplete).
bool build_core(std::string& o, const PodSpans& S, const std::string& env_json, int extra = 0,
                const std::string* tz_utc = nullptr) {
    o.clear();
    o.append("{\"name\":");
    raw_or_null(o, S.name);
    o.append(",\"namespace\":");
    raw_or_null(o, S.ns);
    o.append(",\"uid\":");
    raw_or_null(o, S.uid);
    o.append(",\"environment\":");
    o.append(env_json);
    o.append(",\"status\":{\"phase\":");
    if (S.status_present) {
        raw_or_null(o, S.phase);
        o.append(",\"conditions\":[");
        bool first = true;
        for (const auto& c : S.conditions) {
            if (!first) o.push_back(',');
            first = false;
            o.append("{\"type\":");
            raw_or_null(o, c.type);
            o.append(",\"status\":");
            raw_or_null(o, c.status);
            o.append(",\"reason\":");
            raw_or_null(o, c.reason);
            o.append(",\"message\":");
            raw_or_null(o, c.message);
            o.push_back('}');
        }
        o.append("],\"container_statuses\":[");
        first = true;
        for (const auto& c : S.cstatuses) {
            if (!first) o.push_back(',');
            first = false;
            o.append("{\"name\":");
            raw_or_null(o, c.name);
            o.append(",\"ready\":");
            raw_or_null(o, c.ready);
            o.append(",\"restart_count\":");
            raw_or_null(o, c.restart_count);
            o.append(",\"state\":");
            if (tz_utc) {
                if (!state_repr_json(o, c.state, *tz_utc)) return false;
            } else {
                raw_or_null(o, c.state);
            }
            o.push_back('}');
        }
        o.append("]}");
    } else {
        o.append("\"Unknown\",\"conditions\":[],\"container_statuses\":[]}");
    }
    o.append(",\"spec\":{\"node_name\":");
    if (S.spec_present) {
        raw_or_null(o, S.node_name);
        o.append(",\"containers\":[");
        bool first = true;
        for (const auto& c : S.containers) {
            if (!first) o.push_back(',');
            first = false;
            o.append("{\"name\":");
            raw_or_null(o, c.name);
            o.append(",\"image\":");
            raw_or_null(o, c.image);
            o.push_back('}');
        }
        o.append("]}");
    } else {
        o.append("null,\"containers\":[]}");
    }
    o.append(",\"metadata\":{\"labels\":");
    if (falsy_token(S.labels)) o.append("{}"); else o.append(S.labels.p, S.labels.n);
    o.append(",\"annotations\":");
    if (falsy_token(S.annotations)) o.append("{}"); else o.append(S.annotations.p, S.annotations.n);
    o.append(",\"creation_timestamp\":");
    creation_time(o, S.ctime);
    o.push_back('}');
    if (extra) {
        static const char* names[6] = {"pod_ip", "host_ip", "start_time", "qos_class", "resource_version",
                                       "owner_references"};
        const Span* vals[6] = {&S.pod_ip, &S.host_ip, &S.start_time, &S.qos, &S.rv, &S.owners};
        o.append(",\"extra\":{");
        bool first = true;
        for (int i = 0; i < 6; ++i) {
            if (!(extra >> i & 1)) continue;
            if (!first) o.push_back(',');
            first = false;
            o.push_back('"');
            o.append(names[i]);
            o.append("\":");
            raw_or_null(o, *vals[i]);
        }
        o.push_back('}');
    }
    o.push_back('}');
    return true;
}

#include "validate.inc"

// ----------------------------------------------------------------------------- Python glue

PyObject* g_json_loads = nullptr;
// WatchList (sendInitialEvents=true): the BOOKMARK that ends the initial
// state carries metadata.annotations["k8s.io/initial-events-end"] == "true".
bool initial_events_end(const Span& annotations) {
    if (!annotations.present() || annotations.n < 2 || annotations.p[0] != '{') return false;
    bool found = false;
    try {
        Parser P(annotations.p, annotations.p + annotations.n);
        P.object([&](const char* k, size_t kn) {
            Span v = P.value();
            if (KEYIS("k8s.io/initial-events-end") && v.n == 6 && !std::memcmp(v.p, "\"true\"", 6)) found = true;
        });
    } catch (const ParseError&) {
        return false;
    }
    return found;
}

PyObject* g_types[6];  // ADDED MODIFIED DELETED BOOKMARK ERROR INVALID
enum { T_ADDED, T_MODIFIED, T_DELETED, T_BOOKMARK, T_ERROR, T_INVALID };

void append_utf8_codepoint(std::string& o, uint32_t cp) {
    if (cp < 0x80) {
        o.push_back((char)cp);
    } else if (cp < 0x800) {
        o.push_back((char)(0xC0 | (cp >> 6)));
        o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
        o.push_back((char)(0xE0 | (cp >> 12)));
        o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
        o.push_back((char)(0xF0 | (cp >> 18)));
        o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (cp & 0x3F)));
    }
}

int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

bool read_u4(const char* p, const char* e, uint32_t& out) {
    if (e - p < 4) return false;
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
        int h = hexval(p[i]);
        if (h < 0) return false;
        v = (v << 4) | (uint32_t)h;
    }
    out = v;
    return true;
}

// JSON string token → Python str; non-string / absent → None (new reference).
PyObject* span_to_str(const Span& s) {
    if (!s.is_string()) Py_RETURN_NONE;
    const char* p = s.p + 1;
    size_t n = s.n - 2;
    if (!std::memchr(p, '\\', n)) return PyUnicode_DecodeUTF8(p, (Py_ssize_t)n, "replace");
    std::string o;
    o.reserve(n);
    const char* e = p + n;
    while (p < e) {
        char c = *p++;
        if (c != '\\') {
            o.push_back(c);
            continue;
        }
        if (p >= e) break;
        char d = *p++;
        switch (d) {
            case '"': o.push_back('"'); break;
            case '\\': o.push_back('\\'); break;
            case '/': o.push_back('/'); break;
            case 'b': o.push_back('\b'); break;
            case 'f': o.push_back('\f'); break;
            case 'n': o.push_back('\n'); break;
            case 'r': o.push_back('\r'); break;
            case 't': o.push_back('\t'); break;
            case 'u': {
                uint32_t cp;
                if (!read_u4(p, e, cp)) { o.push_back('?'); break; }
                p += 4;
                if (cp >= 0xD800 && cp <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                    uint32_t lo;
                    if (read_u4(p + 2, e, lo) && lo >= 0xDC00 && lo <= 0xDFFF) {
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        p += 6;
                    }
                }
                append_utf8_codepoint(o, cp);
                break;
            }
            default: o.push_back(d);
        }
    }
    return PyUnicode_DecodeUTF8(o.data(), (Py_ssize_t)o.size(), "surrogatepass");
}

#include "pyrepr.inc"

struct InternTable {
    std::unordered_map<std::string, PyObject*> map;
    ~InternTable() {
        for (auto& kv : map) Py_XDECREF(kv.second);
    }
    // Small-cardinality strings (namespaces, phases): reuse one object.
    PyObject* get(const Span& s) {
        if (!s.is_string() || s.n > 66 || std::memchr(s.p, '\\', s.n)) return span_to_str(s);
        std::string key(s.p + 1, s.n - 2);
        auto it = map.find(key);
        if (it != map.end()) {
            Py_INCREF(it->second);
            return it->second;
        }
        PyObject* v = span_to_str(s);
        if (!v) return nullptr;
        if (map.size() < 4096) {
            Py_INCREF(v);
            map.emplace(std::move(key), v);
        }
        return v;
    }
};

struct DecoderObject {
    PyObject_HEAD
    std::string* partial;
    std::string* env_json;
    std::string* out;
    PodSpans* spans;
    InternTable* interned;
    std::string* chunk_line;  // partial chunk-size / trailer line
    int cstate;               // chunked-framing state (CS_*)
    size_t cremain;           // bytes left in the current chunk
    long long n_events;
    long long n_bytes;
    int extra;  // watcher.payload_extra_fields mask
    int validate;  // watcher.validate: 0 off, 1 payload (default), 2 full
    std::string* tz_utc;     // state_format python_repr (pyrepr.inc); NULL: structured
    PyObject* repr_fallback; // object bytes -> core bytes, for states pyrepr.inc leaves to Python
};

int hexval(char c);

PyObject* make_invalid(const char* why, const char* line, size_t n) {
    PyObject* msg = PyUnicode_FromFormat("%s: %.200s", why, std::string(line, n < 200 ? n : 200).c_str());
    if (!msg) {
        PyErr_Clear();
        msg = PyUnicode_FromString(why);
    }
    PyObject* t = PyTuple_New(9);
    Py_INCREF(g_types[T_INVALID]);
    PyTuple_SET_ITEM(t, 0, g_types[T_INVALID]);
    for (int i = 1; i < 8; ++i) {
        PyObject* v = (i == 6) ? Py_False : Py_None;
        Py_INCREF(v);
        PyTuple_SET_ITEM(t, i, v);
    }
    PyTuple_SET_ITEM(t, 8, msg);
    return t;
}

int type_index(const Span& s) {
    if (!s.is_string()) return -1;
    const char* p = s.p + 1;
    size_t n = s.n - 2;
    if (n == 5 && !std::memcmp(p, "ADDED", 5)) return T_ADDED;
    if (n == 8 && !std::memcmp(p, "MODIFIED", 8)) return T_MODIFIED;
    if (n == 7 && !std::memcmp(p, "DELETED", 7)) return T_DELETED;
    if (n == 8 && !std::memcmp(p, "BOOKMARK", 8)) return T_BOOKMARK;
    if (n == 5 && !std::memcmp(p, "ERROR", 5)) return T_ERROR;
    return -2;  // unknown type string
}

// Build the event tuple for a parsed pod. `tidx` is the event type index.
PyObject* event_tuple(DecoderObject* self, int tidx, PyObject* type_obj, const Span& obj_span) {
    PodSpans& S = *self->spans;
    PyObject* t = PyTuple_New(9);
    if (!t) return nullptr;
    Py_INCREF(type_obj);
    PyTuple_SET_ITEM(t, 0, type_obj);
    if (tidx == T_ERROR) {
        for (int i = 1; i < 8; ++i) {
            PyObject* v = (i == 6) ? Py_False : Py_None;
            Py_INCREF(v);
            PyTuple_SET_ITEM(t, i, v);
        }
        PyObject* raw = PyBytes_FromStringAndSize(obj_span.p, (Py_ssize_t)obj_span.n);
        PyObject* st = raw ? PyObject_CallOneArg(g_json_loads, raw) : nullptr;
        Py_XDECREF(raw);
        if (!st) {
            PyErr_Clear();
            st = PyDict_New();
        }
        PyTuple_SET_ITEM(t, 8, st);
        return t;
    }
    PyObject* uid = span_to_str(S.uid);
    PyObject* ns = self->interned->get(S.ns);
    PyObject* name = span_to_str(S.name);
    PyObject* rv = span_to_str(S.rv);
    PyObject* phase = S.status_present ? self->interned->get(S.phase) : (Py_INCREF(Py_None), Py_None);
    if (!uid || !ns || !name || !rv || !phase) {
        Py_XDECREF(uid); Py_XDECREF(ns); Py_XDECREF(name); Py_XDECREF(rv); Py_XDECREF(phase);
        Py_DECREF(t);
        return nullptr;
    }
    PyTuple_SET_ITEM(t, 1, uid);
    PyTuple_SET_ITEM(t, 2, ns);
    PyTuple_SET_ITEM(t, 3, name);
    PyTuple_SET_ITEM(t, 4, rv);
    PyTuple_SET_ITEM(t, 5, phase);
    PyObject* hs = S.status_present ? Py_True : Py_False;
    Py_INCREF(hs);
    PyTuple_SET_ITEM(t, 6, hs);
    if (tidx == T_BOOKMARK || tidx < 0) {
        Py_INCREF(Py_None);
        PyTuple_SET_ITEM(t, 7, Py_None);
        if (tidx == T_BOOKMARK) {  // extra: True on the WatchList end-of-initial-events marker
            PyObject* end = initial_events_end(S.annotations) ? Py_True : Py_False;
            Py_INCREF(end);
            PyTuple_SET_ITEM(t, 8, end);
            return t;
        }
    } else {
        if (self->validate == 1) {  // no malformed sub-tree into a payload (validate.inc)
            if (const char* why = payload_spans_invalid(S)) {
                Py_DECREF(t);
                return make_invalid(why, obj_span.p, obj_span.n);
            }
        }
        PyObject* core;
        if (build_core(*self->out, S, *self->env_json, self->extra, self->tz_utc)) {
            core = PyBytes_FromStringAndSize(self->out->data(), (Py_ssize_t)self->out->size());
        } else {  // a container state the native repr leaves to models/payload.py
            PyObject* raw = self->repr_fallback ? PyBytes_FromStringAndSize(obj_span.p, (Py_ssize_t)obj_span.n)
                                                : nullptr;
            core = raw ? PyObject_CallOneArg(self->repr_fallback, raw) : nullptr;
            Py_XDECREF(raw);
            if (!core || !PyBytes_Check(core)) {
                PyErr_Clear();
                Py_XDECREF(core);
                Py_DECREF(t);
                return make_invalid("container state not representable", obj_span.p, obj_span.n);
            }
        }
        if (!core) {
            Py_DECREF(t);
            return nullptr;
        }
        PyTuple_SET_ITEM(t, 7, core);
    }
    Py_INCREF(Py_None);
    PyTuple_SET_ITEM(t, 8, Py_None);
    return t;
}

// Decode one watch line. Returns a new tuple, or nullptr with a Python error set.
PyObject* decode_line(DecoderObject* self, const char* b, size_t n) {
    PodSpans& S = *self->spans;
    S.clear();
    if (self->validate == 2) {
        if (const char* why = json_invalid(b, n)) return make_invalid(why, b, n);
    }
    Span type_span, obj_span;
    try {
        Parser P(b + (has_bom(b, n) ? 3 : 0), b + n);  // as json.loads(bytes): 'utf-8-sig'
        P.object([&](const char* k, size_t kn) {
            if (KEYIS("type")) {
                type_span = P.value();
            } else if (KEYIS("object")) {
                if (P.peek() != '{') throw ParseError{"object is not a JSON object"};
                const char* start = P.p_;
                S.clear();  // a repeated "object" key: the last one is the pod
                parse_pod(P, S);
                obj_span.p = start;
                obj_span.n = (size_t)(P.p_ - start);
            } else {
                P.value();
            }
        });
        P.ws();
        if (P.p_ != P.end_) throw ParseError{"trailing data"};
    } catch (const ParseError& e) {
        return make_invalid(e.msg, b, n);
    }
    int tidx = type_index(type_span);
    if (tidx == -1 || !obj_span.present()) return make_invalid("missing type or object", b, n);
    PyObject* type_obj;
    if (tidx >= 0) {
        type_obj = g_types[tidx];
        Py_INCREF(type_obj);
    } else {
        type_obj = span_to_str(type_span);
        if (!type_obj) return nullptr;
    }
    PyObject* t = event_tuple(self, tidx, type_obj, obj_span);
    Py_DECREF(type_obj);
    self->n_events++;
    return t;
}

// ----------------------------------------------------------------------------- methods

int Decoder_init(DecoderObject* self, PyObject* args, PyObject* kwds) {
    static const char* kwlist[] = {"environment", "state_format", nullptr};
    const char* env = nullptr;
    Py_ssize_t envn = 0;
    const char* sf = "structured";
    if (!PyArg_ParseTupleAndKeywords(args, kwds, "s#|s", (char**)kwlist, &env, &envn, &sf)) return -1;
    if (std::strcmp(sf, "structured") != 0 && std::strcmp(sf, "python_repr") != 0) {
        PyErr_SetString(PyExc_ValueError, "state_format must be 'structured' or 'python_repr'");
        return -1;
    }
    delete self->tz_utc;
    self->tz_utc = std::strcmp(sf, "python_repr") == 0 ? new std::string("tzutc()") : nullptr;
    // environment as a JSON string literal (via json.dumps for exact escaping)
    PyObject* envs = PyUnicode_FromStringAndSize(env, envn);
    if (!envs) return -1;
    PyObject* mod = PyImport_ImportModule("json");
    PyObject* dumped = mod ? PyObject_CallMethod(mod, "dumps", "O", envs) : nullptr;
    Py_XDECREF(mod);
    Py_DECREF(envs);
    if (!dumped) return -1;
    Py_ssize_t dn;
    const char* d = PyUnicode_AsUTF8AndSize(dumped, &dn);
    if (!d) {
        Py_DECREF(dumped);
        return -1;
    }
    self->env_json->assign(d, (size_t)dn);
    Py_DECREF(dumped);
    return 0;
}

PyObject* Decoder_new(PyTypeObject* type, PyObject*, PyObject*) {
    DecoderObject* self = (DecoderObject*)type->tp_alloc(type, 0);
    if (!self) return nullptr;
    self->partial = new std::string();
    self->env_json = new std::string("\"\"");
    self->out = new std::string();
    self->out->reserve(8192);
    self->spans = new PodSpans();
    self->interned = new InternTable();
    self->chunk_line = new std::string();
    self->cstate = 0;
    self->cremain = 0;
    self->n_events = 0;
    self->n_bytes = 0;
    self->validate = 1;
    self->tz_utc = nullptr;
    self->repr_fallback = nullptr;
    return (PyObject*)self;
}

void Decoder_dealloc(DecoderObject* self) {
    delete self->partial;
    delete self->env_json;
    delete self->out;
    delete self->spans;
    delete self->interned;
    delete self->chunk_line;
    delete self->tz_utc;
    Py_XDECREF(self->repr_fallback);
    Py_TYPE(self)->tp_free((PyObject*)self);
}

bool blank(const char* b, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (!(b[i] == ' ' || b[i] == '\r' || b[i] == '\t' || b[i] == '\n')) return false;
    return true;
}

// Split `data` into NDJSON lines (carrying a partial line across calls) and
// append one event tuple per complete non-blank line to `out`.
bool process_segment(DecoderObject* self, const char* data, size_t n, PyObject* out) {
    std::string& partial = *self->partial;
    size_t pos = 0;
    auto emit = [&](const char* b, size_t len) -> bool {
        if (len == 0 || blank(b, len)) return true;
        PyObject* t = decode_line(self, b, len);
        if (!t) return false;
        int r = PyList_Append(out, t);
        Py_DECREF(t);
        return r == 0;
    };
    if (!partial.empty()) {
        const char* nl = (const char*)std::memchr(data, '\n', n);
        if (!nl) {
            partial.append(data, n);
            return true;
        }
        partial.append(data, (size_t)(nl - data));
        bool ok = emit(partial.data(), partial.size());
        partial.clear();
        if (!ok) return false;
        pos = (size_t)(nl - data) + 1;
    }
    while (pos < n) {
        const char* nl = (const char*)std::memchr(data + pos, '\n', n - pos);
        if (!nl) {
            partial.assign(data + pos, n - pos);
            break;
        }
        if (!emit(data + pos, (size_t)(nl - (data + pos)))) return false;
        pos = (size_t)(nl - data) + 1;
    }
    return true;
}

PyObject* Decoder_feed(DecoderObject* self, PyObject* arg) {
    Py_buffer view;
    if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
    self->n_bytes += (long long)view.len;
    PyObject* out = PyList_New(0);
    if (out && !process_segment(self, (const char*)view.buf, (size_t)view.len, out)) {
        Py_DECREF(out);
        out = nullptr;
    }
    PyBuffer_Release(&view);
    return out;
}

// HTTP/1.1 chunked transfer framing, decoded in place of the Python parser
// for the watch stream: size line → data → CRLF ... → 0-size chunk → trailers.
enum { CS_SIZE, CS_DATA, CS_DATA_END, CS_TRAILER, CS_DONE };

bool parse_chunk_size(const std::string& line, size_t& size) {
    size_t v = 0;
    size_t i = 0, n = line.size();
    while (i < n && (line[i] == ' ' || line[i] == '\t')) ++i;
    size_t start = i;
    for (; i < n; ++i) {
        int h = hexval(line[i]);
        if (h < 0) break;
        if (v > (SIZE_MAX >> 4)) return false;
        v = (v << 4) | (size_t)h;
    }
    if (i == start) return false;
    while (i < n && (line[i] == ' ' || line[i] == '\t' || line[i] == '\r')) ++i;
    if (i < n && line[i] != ';') return false;
    size = v;
    return true;
}

PyObject* Decoder_feed_chunked(DecoderObject* self, PyObject* arg) {
    Py_buffer view;
    if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
    const char* data = (const char*)view.buf;
    size_t n = (size_t)view.len;
    self->n_bytes += (long long)n;
    PyObject* out = PyList_New(0);
    if (!out) {
        PyBuffer_Release(&view);
        return nullptr;
    }
    std::string& line = *self->chunk_line;
    size_t i = 0;
    bool ok = true;
    while (ok && i < n && self->cstate != CS_DONE) {
        switch (self->cstate) {
            case CS_SIZE: {
                const char* nl = (const char*)std::memchr(data + i, '\n', n - i);
                if (!nl) {
                    line.append(data + i, n - i);
                    if (line.size() > 4096) {
                        PyErr_SetString(PyExc_ValueError, "chunk size line too long");
                        ok = false;
                    }
                    i = n;
                    break;
                }
                line.append(data + i, (size_t)(nl - (data + i)));
                i = (size_t)(nl - data) + 1;
                size_t size;
                if (!parse_chunk_size(line, size)) {
                    PyErr_Format(PyExc_ValueError, "bad chunk size line %.40s", line.c_str());
                    ok = false;
                    break;
                }
                line.clear();
                if (size == 0) {
                    self->cstate = CS_TRAILER;
                } else {
                    self->cremain = size;
                    self->cstate = CS_DATA;
                }
                break;
            }
            case CS_DATA: {
                size_t take = self->cremain < n - i ? self->cremain : n - i;
                ok = process_segment(self, data + i, take, out);
                i += take;
                self->cremain -= take;
                if (self->cremain == 0) self->cstate = CS_DATA_END;
                break;
            }
            case CS_DATA_END: {
                const char* nl = (const char*)std::memchr(data + i, '\n', n - i);
                if (!nl) {
                    i = n;
                    break;
                }
                i = (size_t)(nl - data) + 1;
                self->cstate = CS_SIZE;
                break;
            }
            case CS_TRAILER: {
                const char* nl = (const char*)std::memchr(data + i, '\n', n - i);
                if (!nl) {
                    line.append(data + i, n - i);
                    i = n;
                    break;
                }
                line.append(data + i, (size_t)(nl - (data + i)));
                i = (size_t)(nl - data) + 1;
                bool empty = line.empty() || (line.size() == 1 && line[0] == '\r');
                line.clear();
                if (empty) self->cstate = CS_DONE;
                break;
            }
        }
    }
    PyBuffer_Release(&view);
    if (!ok) {
        Py_DECREF(out);
        return nullptr;
    }
    return out;
}

PyObject* Decoder_body_done(DecoderObject* self, PyObject*) {
    return PyBool_FromLong(self->cstate == CS_DONE);
}

PyObject* Decoder_reset(DecoderObject* self, PyObject*) {
    self->partial->clear();
    self->chunk_line->clear();
    self->cstate = CS_SIZE;
    self->cremain = 0;
    Py_RETURN_NONE;
}

// decode_list(body) -> (resourceVersion, continue, [ADDED tuples])
PyObject* Decoder_decode_list(DecoderObject* self, PyObject* arg) {
    Py_buffer view;
    if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
    const char* b = (const char*)view.buf;
    size_t n = (size_t)view.len;
    if (self->validate == 2) {
        if (const char* why = json_invalid(b, n)) {
            PyBuffer_Release(&view);
            PyErr_Format(PyExc_ValueError, "invalid list body: %s", why);
            return nullptr;
        }
    }
    PyObject* items = PyList_New(0);
    Span rv, cont;
    bool failed = false;
    try {
        Parser P(b, b + n);
        P.object([&](const char* k, size_t kn) {
            if (KEYIS("metadata")) {
                if (P.null_here()) return;
                P.object([&](const char* k2, size_t kn2) {
                    const char* k = k2; size_t kn = kn2;
                    if (KEYIS("resourceVersion")) rv = P.value();
                    else if (KEYIS("continue")) cont = P.value();
                    else P.value();
                });
            } else if (KEYIS("items")) {
                if (P.null_here()) return;
                P.array([&]() {
                    if (failed) { P.value(); return; }
                    if (P.peek() != '{') { P.value(); return; }
                    self->spans->clear();
                    const char* start = P.p_;
                    parse_pod(P, *self->spans);
                    Span obj;
                    obj.p = start;
                    obj.n = (size_t)(P.p_ - start);
                    PyObject* t = event_tuple(self, T_ADDED, g_types[T_ADDED], obj);
                    if (!t || PyList_Append(items, t) < 0) failed = true;
                    Py_XDECREF(t);
                    self->n_events++;
                });
            } else {
                P.value();
            }
        });
    } catch (const ParseError& e) {
        PyBuffer_Release(&view);
        Py_DECREF(items);
        PyErr_Format(PyExc_ValueError, "invalid list body: %s", e.msg);
        return nullptr;
    }
    PyBuffer_Release(&view);
    if (failed) {
        Py_DECREF(items);
        return nullptr;
    }
    PyObject* rvo = span_to_str(rv);
    PyObject* co = span_to_str(cont);
    if (co && PyUnicode_Check(co) && PyUnicode_GET_LENGTH(co) == 0) {
        Py_DECREF(co);
        Py_INCREF(Py_None);
        co = Py_None;
    }
    PyObject* res = Py_BuildValue("(NNN)", rvo, co, items);
    return res;
}

PyObject* Decoder_core(DecoderObject*, PyObject* ev) {
    if (!PyTuple_Check(ev) || PyTuple_GET_SIZE(ev) < 8) {
        PyErr_SetString(PyExc_TypeError, "expected an event tuple");
        return nullptr;
    }
    PyObject* c = PyTuple_GET_ITEM(ev, 7);
    Py_INCREF(c);
    return c;
}

// core_from_summary(uid, ns, name, phase) -> bytes: payload core for a pod
// known only from the cache (synthesised DELETED after a relist).
PyObject* Decoder_core_from_summary(DecoderObject* self, PyObject* args) {
    PyObject *uid, *ns, *name, *phase;
    if (!PyArg_ParseTuple(args, "OOOO", &uid, &ns, &name, &phase)) return nullptr;
    PyObject* mod = PyImport_ImportModule("json");
    if (!mod) return nullptr;
    PyObject* dumps = PyObject_GetAttrString(mod, "dumps");
    Py_DECREF(mod);
    if (!dumps) return nullptr;
    std::string buf[4];
    PyObject* vals[4] = {uid, ns, name, phase};
    for (int i = 0; i < 4; ++i) {
        PyObject* kw = Py_BuildValue("{s:O}", "ensure_ascii", Py_False);
        PyObject* a = PyTuple_Pack(1, vals[i]);
        PyObject* r = (kw && a) ? PyObject_Call(dumps, a, kw) : nullptr;
        Py_XDECREF(kw);
        Py_XDECREF(a);
        if (!r) {
            Py_DECREF(dumps);
            return nullptr;
        }
        Py_ssize_t ln;
        const char* s = PyUnicode_AsUTF8AndSize(r, &ln);
        buf[i].assign(s, (size_t)ln);
        Py_DECREF(r);
    }
    Py_DECREF(dumps);
    PodSpans S;
    S.meta_present = true;
    S.uid = Span{buf[0].data(), buf[0].size()};
    S.ns = Span{buf[1].data(), buf[1].size()};
    S.name = Span{buf[2].data(), buf[2].size()};
    if (phase != Py_None) {
        S.status_present = true;
        S.phase = Span{buf[3].data(), buf[3].size()};
    }
    build_core(*self->out, S, *self->env_json, self->extra);
    return PyBytes_FromStringAndSize(self->out->data(), (Py_ssize_t)self->out->size());
}

// set_repr(tz_utc_repr, fallback): python_repr details (engine/pipeline.py::repr_settings)
PyObject* Decoder_set_repr(DecoderObject* self, PyObject* args) {
    const char* tz;
    PyObject* fn;
    if (!PyArg_ParseTuple(args, "sO", &tz, &fn)) return nullptr;
    if (!self->tz_utc) {
        PyErr_SetString(PyExc_ValueError, "set_repr: the decoder is not in python_repr mode");
        return nullptr;
    }
    *self->tz_utc = tz;
    Py_INCREF(fn);
    Py_XSETREF(self->repr_fallback, fn);
    Py_RETURN_NONE;
}

PyObject* Decoder_set_validate(DecoderObject* self, PyObject* arg) {
    long v = PyLong_AsLong(arg);
    if (PyErr_Occurred()) return nullptr;
    if (v < 0 || v > 2) {
        PyErr_SetString(PyExc_ValueError, "validate mode must be 0, 1 or 2");
        return nullptr;
    }
    self->validate = (int)v;
    Py_RETURN_NONE;
}

PyObject* Decoder_set_extra(DecoderObject* self, PyObject* arg) {
    self->extra = (int)PyLong_AsLong(arg);
    if (PyErr_Occurred()) return nullptr;
    Py_RETURN_NONE;
}

PyObject* Decoder_stats(DecoderObject* self, PyObject*) {
    return Py_BuildValue("{s:L,s:L}", "events", self->n_events, "bytes", self->n_bytes);
}

PyMethodDef Decoder_methods[] = {
    {"set_extra", (PyCFunction)Decoder_set_extra, METH_O, "set_extra(mask): watcher.payload_extra_fields"},
    {"set_validate", (PyCFunction)Decoder_set_validate, METH_O, "set_validate(0 off | 1 payload | 2 full)"},
    {"set_repr", (PyCFunction)Decoder_set_repr, METH_VARARGS, "set_repr(tz_utc_repr, fallback): python_repr"},
    {"feed", (PyCFunction)Decoder_feed, METH_O, "feed(bytes) -> list of event tuples"},
    {"feed_chunked", (PyCFunction)Decoder_feed_chunked, METH_O,
     "feed_chunked(bytes) -> events; input keeps its HTTP chunked framing"},
    {"body_done", (PyCFunction)Decoder_body_done, METH_NOARGS, "True after the terminating 0-size chunk"},
    {"reset", (PyCFunction)Decoder_reset, METH_NOARGS, "drop partial line and chunk state"},
    {"decode_list", (PyCFunction)Decoder_decode_list, METH_O, "decode_list(body) -> (rv, continue, events)"},
    {"core", (PyCFunction)Decoder_core, METH_O, "core(event) -> payload core bytes"},
    {"core_from_summary", (PyCFunction)Decoder_core_from_summary, METH_VARARGS,
     "core_from_summary(uid, ns, name, phase) -> bytes"},
    {"stats", (PyCFunction)Decoder_stats, METH_NOARGS, "counters"},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject DecoderType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// ----------------------------------------------------------------------------- ResponseScanner
//
// HTTP/1.1 response framing for the clusterapi notifier pool: one feed() per
// socket read returns every complete response in it. A 2xx keep-alive
// response is returned as its int status (no allocation); anything else as
// (status, keep_alive, body) so the pool can log / close. Handles
// Content-Length, chunked bodies, 1xx/204/304 and read-until-close framing.

struct ScannerObject {
    PyObject_HEAD
    std::string* buf;
    size_t pos;
};

bool ieq_prefix(const char* p, const char* e, const char* lit) {
    size_t n = std::strlen(lit);
    if ((size_t)(e - p) < n) return false;
    for (size_t i = 0; i < n; ++i) {
        char c = p[i];
        if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
        if (c != lit[i]) return false;
    }
    return true;
}

bool contains_token_ci(const char* p, const char* e, const char* tok) {
    size_t n = std::strlen(tok);
    for (const char* q = p; q + n <= e; ++q)
        if (ieq_prefix(q, e, tok)) return true;
    return false;
}

// Retry-After: <delta-seconds> (fractions accepted, capped at 300 s); -1 when
// absent or an HTTP-date (which clusterapi-style services do not send).
double parse_retry_after(const char* v, const char* e) {
    while (v < e && (*v == ' ' || *v == '\t')) ++v;
    if (v >= e || !is_digit(*v)) return -1.0;
    double secs = 0.0;
    while (v < e && is_digit(*v)) secs = secs * 10.0 + (*v++ - '0');
    if (v < e && *v == '.') {
        double scale = 0.1;
        for (++v; v < e && is_digit(*v); ++v, scale *= 0.1) secs += (*v - '0') * scale;
    }
    while (v < e && (*v == ' ' || *v == '\t')) ++v;
    if (v != e) return -1.0;
    return secs > 300.0 ? 300.0 : secs;
}

// Try to parse one complete response at b[0..n). Returns bytes consumed (0 =
// incomplete, SIZE_MAX = malformed); fills status, keep_alive, body span and
// retry_after (seconds, -1 = no Retry-After header).
size_t scan_response(const char* b, size_t n, int& status, bool& keep_alive, std::string& body,
                     bool& until_close, double& retry_after) {
    const char* e = b + n;
    const char* he = nullptr;
    for (const char* q = b; q + 3 < e; ++q) {
        q = (const char*)std::memchr(q, '\r', (size_t)(e - q));
        if (!q || q + 3 >= e) break;
        if (q[1] == '\n' && q[2] == '\r' && q[3] == '\n') {
            he = q;
            break;
        }
    }
    if (!he) return n > 65536 ? SIZE_MAX : 0;
    if (n < 12 || std::memcmp(b, "HTTP/1.", 7) != 0) return SIZE_MAX;
    bool http10 = b[7] == '0';
    const char* sp = (const char*)std::memchr(b, ' ', (size_t)(he - b));
    if (!sp || he - sp < 4) return SIZE_MAX;
    status = 0;
    for (int i = 1; i <= 3; ++i) {
        if (!is_digit(sp[i])) return SIZE_MAX;
        status = status * 10 + (sp[i] - '0');
    }
    long long clen = -1;
    retry_after = -1.0;
    bool chunked = false, conn_close = false, conn_keep = false;
    const char* line = (const char*)std::memchr(b, '\n', (size_t)(he - b));
    while (line && line < he) {
        const char* ls = line + 1;
        const char* le = (const char*)std::memchr(ls, '\r', (size_t)(he + 2 - ls));
        if (!le) le = he;
        if (ieq_prefix(ls, le, "content-length:")) {
            const char* v = ls + 15;
            while (v < le && (*v == ' ' || *v == '\t')) ++v;
            clen = 0;
            while (v < le && is_digit(*v)) clen = clen * 10 + (*v++ - '0');
        } else if (ieq_prefix(ls, le, "transfer-encoding:")) {
            chunked = contains_token_ci(ls + 18, le, "chunked");
        } else if (ieq_prefix(ls, le, "connection:")) {
            conn_close = contains_token_ci(ls + 11, le, "close");
            conn_keep = contains_token_ci(ls + 11, le, "keep-alive");
        } else if (ieq_prefix(ls, le, "retry-after:")) {
            retry_after = parse_retry_after(ls + 12, le);
        }
        line = (const char*)std::memchr(ls, '\n', (size_t)(he + 2 - ls));
        if (line && line >= he) break;
    }
    keep_alive = http10 ? conn_keep : !conn_close;
    const char* bs = he + 4;
    body.clear();
    until_close = false;
    if ((status >= 100 && status < 200) || status == 204 || status == 304) return (size_t)(bs - b);
    if (chunked) {
        const char* q = bs;
        while (true) {
            const char* nl = (const char*)std::memchr(q, '\n', (size_t)(e - q));
            if (!nl) return 0;
            size_t sz = 0;
            const char* h = q;
            int digits = 0;
            while (h < nl && hexval(*h) >= 0) {
                sz = (sz << 4) | (size_t)hexval(*h++);
                ++digits;
            }
            if (!digits) return SIZE_MAX;
            q = nl + 1;
            if (sz == 0) {
                while (true) {  // trailers up to the empty line
                    const char* t = (const char*)std::memchr(q, '\n', (size_t)(e - q));
                    if (!t) return 0;
                    bool empty = (t == q) || (t == q + 1 && *q == '\r');
                    q = t + 1;
                    if (empty) return (size_t)(q - b);
                }
            }
            if ((size_t)(e - q) < sz + 2) return 0;
            body.append(q, sz);
            q += sz;
            const char* crlf = (const char*)std::memchr(q, '\n', (size_t)(e - q));
            if (!crlf) return 0;
            q = crlf + 1;
        }
    }
    if (clen >= 0) {
        if ((size_t)(e - bs) < (size_t)clen) return 0;
        body.assign(bs, (size_t)clen);
        return (size_t)(bs - b) + (size_t)clen;
    }
    // no framing: body runs to EOF; report what is here and let the caller close
    until_close = true;
    keep_alive = false;
    body.assign(bs, (size_t)(e - bs));
    return n;
}

PyObject* Scanner_new(PyTypeObject* type, PyObject*, PyObject*) {
    ScannerObject* self = (ScannerObject*)type->tp_alloc(type, 0);
    if (!self) return nullptr;
    self->buf = new std::string();
    self->pos = 0;
    return (PyObject*)self;
}

void Scanner_dealloc(ScannerObject* self) {
    delete self->buf;
    Py_TYPE(self)->tp_free((PyObject*)self);
}

PyObject* Scanner_feed(ScannerObject* self, PyObject* arg) {
    Py_buffer view;
    if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
    std::string& buf = *self->buf;
    const char* data;
    size_t n;
    bool direct = buf.empty();
    if (direct) {
        data = (const char*)view.buf;
        n = (size_t)view.len;
    } else {
        buf.append((const char*)view.buf, (size_t)view.len);
        data = buf.data();
        n = buf.size();
    }
    PyObject* out = PyList_New(0);
    std::string body;
    size_t pos = 0;
    bool ok = out != nullptr;
    while (ok && pos < n) {
        int status = 0;
        bool keep = true, until_close = false;
        double retry_after = -1.0;
        size_t used = scan_response(data + pos, n - pos, status, keep, body, until_close, retry_after);
        if (used == 0) break;
        if (used == SIZE_MAX) {
            PyErr_SetString(PyExc_ValueError, "malformed HTTP response");
            ok = false;
            break;
        }
        pos += used;
        PyObject* item;
        if (status >= 200 && status < 300 && keep) {
            item = PyLong_FromLong(status);
        } else {
            item = Py_BuildValue("(iOy#d)", status, keep ? Py_True : Py_False, body.data(),
                                 (Py_ssize_t)body.size(), retry_after);
        }
        if (!item || PyList_Append(out, item) < 0) ok = false;
        Py_XDECREF(item);
        if (until_close) break;
    }
    if (ok) {
        if (direct) {
            if (pos < n) buf.assign(data + pos, n - pos);
        } else {
            buf.erase(0, pos);
        }
    }
    PyBuffer_Release(&view);
    if (!ok) {
        Py_XDECREF(out);
        return nullptr;
    }
    return out;
}

PyObject* Scanner_reset(ScannerObject* self, PyObject*) {
    self->buf->clear();
    Py_RETURN_NONE;
}

PyObject* Scanner_pending(ScannerObject* self, PyObject*) {
    return PyLong_FromSize_t(self->buf->size());
}

PyMethodDef Scanner_methods[] = {
    {"feed", (PyCFunction)Scanner_feed, METH_O,
     "feed(bytes) -> [status | (status, keep_alive, body)] for each complete response"},
    {"reset", (PyCFunction)Scanner_reset, METH_NOARGS, "drop buffered bytes"},
    {"pending", (PyCFunction)Scanner_pending, METH_NOARGS, "buffered byte count"},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject ScannerType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// format_event_timestamp(utc: bool) -> str: datetime.now().isoformat() equivalent
// stamp_fields(buf, rv_off, rvs, ndigits, uid_off, uid_text): benchmark
// fixtures (testing/cluster_replay.py) re-stamp a prerendered watch stream per
// step — rvs[i] as ndigits zero-padded decimal digits at buf[rv_off[i]], and
// uid_text at every buf[uid_off[j]] — bounds-checked, in place. The numpy
// version of this was most of the fixture's time at ~1.5M events/s.
PyObject* kw_stamp_fields(PyObject*, PyObject* args) {
    Py_buffer buf, rvo, rvs, uo;
    int nd;
    const char* ut;
    Py_ssize_t un;
    if (!PyArg_ParseTuple(args, "w*y*y*iy*y#", &buf, &rvo, &rvs, &nd, &uo, &ut, &un)) return nullptr;
    bool ok = rvo.len == rvs.len && rvo.len % 8 == 0 && uo.len % 8 == 0 && nd > 0 && nd <= 19;
    const int64_t* ro = (const int64_t*)rvo.buf;
    const int64_t* rv = (const int64_t*)rvs.buf;
    const int64_t* uof = (const int64_t*)uo.buf;
    const size_t n = (size_t)rvo.len / 8, m = (size_t)uo.len / 8, blen = (size_t)buf.len;
    char* b = (char*)buf.buf;
    for (size_t i = 0; ok && i < n; ++i) {
        if (ro[i] < 0 || (size_t)ro[i] + (size_t)nd > blen || rv[i] < 0) {
            ok = false;
            break;
        }
        int64_t v = rv[i];
        for (int d = nd - 1; d >= 0; --d) {
            b[ro[i] + d] = (char)('0' + v % 10);
            v /= 10;
        }
    }
    for (size_t j = 0; ok && j < m; ++j) {
        if (uof[j] < 0 || (size_t)uof[j] + (size_t)un > blen) {
            ok = false;
            break;
        }
        std::memcpy(b + uof[j], ut, (size_t)un);
    }
    PyBuffer_Release(&buf);
    PyBuffer_Release(&rvo);
    PyBuffer_Release(&rvs);
    PyBuffer_Release(&uo);
    if (!ok) {
        PyErr_SetString(PyExc_ValueError, "stamp_fields: offsets out of range or arrays mismatched");
        return nullptr;
    }
    Py_RETURN_NONE;
}

PyObject* kw_event_timestamp(PyObject*, PyObject* arg) {
    int utc = PyObject_IsTrue(arg);
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    struct tm tmv;
    time_t secs = ts.tv_sec;
    if (utc) gmtime_r(&secs, &tmv); else localtime_r(&secs, &tmv);
    long micro = ts.tv_nsec / 1000;
    char buf[64];
    int n = std::snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02d", tmv.tm_year + 1900, tmv.tm_mon + 1,
                          tmv.tm_mday, tmv.tm_hour, tmv.tm_min, tmv.tm_sec);
    if (micro) n += std::snprintf(buf + n, sizeof buf - n, ".%06ld", micro);
    if (utc) n += std::snprintf(buf + n, sizeof buf - n, "+00:00");
    return PyUnicode_FromStringAndSize(buf, n);
}

PyObject* kw_cpu_features(PyObject*, PyObject*) {
#if defined(__x86_64__)
    return Py_BuildValue("{s:O,s:O}", "avx2", Parser::use_avx2 ? Py_True : Py_False, "avx512",
                         Parser::use_avx512 ? Py_True : Py_False);
#else
    return Py_BuildValue("{s:O,s:O}", "avx2", Py_False, "avx512", Py_False);
#endif
}

// set_simd(True) = best supported level, False = scalar, "avx2" = cap at AVX2.
PyObject* kw_set_simd(PyObject*, PyObject* arg) {
#if defined(__x86_64__)
    bool cap_avx2 = PyUnicode_Check(arg) && PyUnicode_CompareWithASCIIString(arg, "avx2") == 0;
    int on = PyObject_IsTrue(arg);
    if (on < 0) return nullptr;
    Parser::use_avx2 = on && simd_supported();
    Parser::use_avx512 = on && !cap_avx2 && avx512_supported();
#endif
    Py_RETURN_NONE;
}

// bench_parse(data, mode, repeat) -> seconds. Times the pure C++ stages on
// newline-separated lines without creating Python objects:
// mode 0 = structural skip of each line, 1 = field extraction (spans),
// 2 = extraction + payload core assembly, 3 = filter-first light extraction,
// 4 = light extraction + materialize + core assembly.
PyObject* kw_bench_parse(PyObject*, PyObject* args) {
    Py_buffer view;
    int mode = 2, repeat = 1;
    if (!PyArg_ParseTuple(args, "y*|ii", &view, &mode, &repeat)) return nullptr;
    const char* b = (const char*)view.buf;
    const char* e = b + view.len;
    std::vector<std::pair<const char*, const char*>> lines;
    for (const char* p = b; p < e;) {
        const char* nl = (const char*)std::memchr(p, '\n', (size_t)(e - p));
        if (!nl) nl = e;
        if (nl > p) lines.emplace_back(p, nl);
        p = nl + 1;
    }
    PodSpans S;
    std::string out;
    out.reserve(8192);
    std::string env = "\"production\"";
    size_t sink = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    try {
        for (int r = 0; r < repeat; ++r) {
            for (auto& ln : lines) {
                Parser P(ln.first, ln.second);
                if (mode == 0) {
                    sink += (size_t)(P.value().n);
                    continue;
                }
                S.clear();
                const bool light = mode >= 3;
                P.object([&](const char* k, size_t kn) {
                    if (KEYIS("object")) {
                        if (light) parse_pod_light(P, S); else parse_pod(P, S);
                    } else {
                        P.value();
                    }
                });
                if (mode == 2 || mode == 4 || mode == 5) {
                    static const std::string tz_utc = "tzutc()";
                    materialize(S);
                    build_core(out, S, env, 0, mode == 5 ? &tz_utc : nullptr);  // 5: state_format python_repr
                    sink += out.size();
                } else {
                    sink += S.name.n;
                }
            }
        }
    } catch (const ParseError& err) {
        PyBuffer_Release(&view);
        PyErr_SetString(PyExc_ValueError, err.msg);
        return nullptr;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    PyBuffer_Release(&view);
    double secs = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return Py_BuildValue("(dn)", secs, (Py_ssize_t)sink);
}

#include "podcache.inc"
#include "logsink.inc"
#include "engine.inc"
#include "checkpoint.inc"
#include "relist.inc"
#include "tls13.inc"
#include "readerhub.inc"
#include "sinkserver.inc"
#include "looplag.inc"

// json_invalid(data) -> None if json.loads(data) accepts it, else the reason (validate.inc)
PyObject* kw_json_invalid(PyObject*, PyObject* arg) {
    Py_buffer view;
    if (PyObject_GetBuffer(arg, &view, PyBUF_SIMPLE) < 0) return nullptr;
    const char* why = json_invalid((const char*)view.buf, (size_t)view.len);
    PyBuffer_Release(&view);
    if (!why) Py_RETURN_NONE;
    return PyUnicode_FromString(why);
}

// bench_validate(data, repeat) -> seconds: json_invalid over every line of data
PyObject* kw_bench_validate(PyObject*, PyObject* args) {
    Py_buffer view;
    int repeat = 1;
    if (!PyArg_ParseTuple(args, "y*|i", &view, &repeat)) return nullptr;
    const char* b = (const char*)view.buf;
    const char* e = b + view.len;
    std::vector<std::pair<const char*, size_t>> lines;
    for (const char* p = b; p < e;) {
        const char* nl = (const char*)std::memchr(p, '\n', (size_t)(e - p));
        if (!nl) nl = e;
        if (nl > p) lines.emplace_back(p, (size_t)(nl - p));
        p = nl + 1;
    }
    size_t bad = 0;
    const int64_t t0 = mono_ns();
    for (int r = 0; r < repeat; ++r)
        for (auto& ln : lines) bad += json_invalid(ln.first, ln.second) != nullptr;
    const int64_t t1 = mono_ns();
    PyBuffer_Release(&view);
    return Py_BuildValue("(dn)", (double)(t1 - t0) * 1e-9, (Py_ssize_t)bad);
}

// malloc_info() -> the C heap (glibc mallinfo2, every arena): bytes in use
// (small chunks + mmapped blocks), free inside the heap (retained, not
// returned to the kernel), and the arenas' size. Memory accounting for the
// watcher's RSS beyond the cache / owed notifications / read buffers.
PyObject* kw_malloc_info(PyObject*, PyObject*) {
    struct mallinfo2 mi = mallinfo2();
    return Py_BuildValue("{s:n,s:n,s:n,s:n}", "in_use_bytes", (Py_ssize_t)(mi.uordblks + mi.hblkhd), "free_bytes",
                         (Py_ssize_t)mi.fordblks, "arena_bytes", (Py_ssize_t)mi.arena, "mmap_bytes",
                         (Py_ssize_t)mi.hblkhd);
}

// malloc_arenas() -> [(arena, free_bytes, system_bytes)]: glibc's
// malloc_info() per arena (0 is the main arena, the event loop's; the others
// belong to native threads) — where the retained free bytes of the C heap sit
// (soak attribution: benchmarks/soak.py samples it).
PyObject* kw_malloc_arenas(PyObject*, PyObject*) {
    char* buf = nullptr;
    size_t len = 0;
    FILE* f = open_memstream(&buf, &len);
    if (!f) return PyErr_SetFromErrno(PyExc_OSError);
    malloc_info(0, f);
    std::fclose(f);
    std::string xml(buf ? buf : "", len);
    std::free(buf);
    PyObject* out = PyList_New(0);
    if (!out) return nullptr;
    auto attr = [](const std::string& x, size_t from, size_t to, const char* tag, const char* key) -> long long {
        const size_t t = x.find(tag, from);
        if (t == std::string::npos || t >= to) return 0;
        const size_t k = x.find(key, t);
        if (k == std::string::npos || k >= to) return 0;
        return std::atoll(x.c_str() + k + std::strlen(key));
    };
    size_t pos = 0;
    for (;;) {
        const size_t h = xml.find("<heap nr=\"", pos);
        if (h == std::string::npos) break;
        const size_t e = xml.find("</heap>", h);
        if (e == std::string::npos) break;
        const int nr = std::atoi(xml.c_str() + h + 10);
        const long long fr = attr(xml, h, e, "<total type=\"fast\"", "size=\"") +
                             attr(xml, h, e, "<total type=\"rest\"", "size=\"");
        const long long sys = attr(xml, h, e, "<system type=\"current\"", "size=\"");
        PyObject* t = Py_BuildValue("(iLL)", nr, fr, sys);
        if (!t || PyList_Append(out, t) < 0) {
            Py_XDECREF(t);
            Py_DECREF(out);
            return nullptr;
        }
        Py_DECREF(t);
        pos = e;
    }
    return out;
}

// malloc_trim() -> bool: give the C heap's free pages back to the kernel
// (every arena; the decode workers' arenas keep what their threads freed).
// Runs without the GIL: the service calls it from an executor thread.
PyObject* kw_malloc_trim(PyObject*, PyObject*) {
    int r;
    Py_BEGIN_ALLOW_THREADS
    r = malloc_trim(0);
    Py_END_ALLOW_THREADS
    return PyBool_FromLong(r);
}

// malloc_tune(mmap_threshold, trim_threshold) -> bool: fixed glibc thresholds.
// Left dynamic, glibc raises its mmap threshold to the size of every large
// block freed (up to 32 MiB), so after one 4 MiB read buffer or relist batch
// goes, later multi-MiB transients are carved from the arenas between
// long-lived chunks and what they free stays there as holes that neither
// trimming nor malloc_trim can return (round-5 soak: RSS +12 MiB, all of it
// retained free bytes). A fixed threshold keeps every block at or above it
// on its own mapping, unmapped when freed. Process-wide; call once at start.
PyObject* kw_malloc_tune(PyObject*, PyObject* args) {
    Py_ssize_t mmap_thr = 0, trim_thr = 0;
    if (!PyArg_ParseTuple(args, "nn", &mmap_thr, &trim_thr)) return nullptr;
    if (mmap_thr <= 0 || trim_thr <= 0 || mmap_thr > (Py_ssize_t)(32 << 20) || trim_thr > ((Py_ssize_t)1 << 30)) {
        PyErr_SetString(PyExc_ValueError, "malloc_tune: thresholds out of range");
        return nullptr;
    }
    const int a = mallopt(M_MMAP_THRESHOLD, (int)mmap_thr);
    const int b = mallopt(M_TRIM_THRESHOLD, (int)trim_thr);
    return PyBool_FromLong(a == 1 && b == 1);
}

PyMethodDef module_methods[] = {
    {"malloc_tune", (PyCFunction)kw_malloc_tune, METH_VARARGS,
     "malloc_tune(mmap_threshold, trim_threshold) -> ok (glibc mallopt; fixes both, disabling their sliding)"},
    {"malloc_trim", (PyCFunction)kw_malloc_trim, METH_NOARGS, "malloc_trim() -> released (glibc malloc_trim(0), no GIL)"},
    {"malloc_arenas", (PyCFunction)kw_malloc_arenas, METH_NOARGS,
     "malloc_arenas() -> [(arena, free_bytes, system_bytes)] (glibc malloc_info per arena)"},
    {"malloc_info", (PyCFunction)kw_malloc_info, METH_NOARGS,
     "malloc_info() -> {in_use_bytes, free_bytes, arena_bytes, mmap_bytes} (glibc mallinfo2)"},
    {"json_invalid", (PyCFunction)kw_json_invalid, METH_O, "json_invalid(data) -> None | reason (json.loads semantics)"},
    {"bench_validate", (PyCFunction)kw_bench_validate, METH_VARARGS, "bench_validate(lines, repeat) -> (seconds, invalid)"},
    {"bench_parse", (PyCFunction)kw_bench_parse, METH_VARARGS, "bench_parse(data, mode=2, repeat=1)"},
    {"event_timestamp", (PyCFunction)kw_event_timestamp, METH_O, "event_timestamp(utc) -> str"},
    {"stamp_fields", (PyCFunction)kw_stamp_fields, METH_VARARGS,
     "stamp_fields(buf, rv_off, rvs, ndigits, uid_off, uid_text): fixture re-stamping (int64 arrays)"},
    {"cpu_features", (PyCFunction)kw_cpu_features, METH_NOARGS, "SIMD paths in use"},
    {"set_simd", (PyCFunction)kw_set_simd, METH_O, "enable/disable the AVX2 scanner"},
    {"apply_stats", (PyCFunction)kw_apply_stats, METH_NOARGS,
     "apply_stats() -> cumulative counts of the partitioned and serial apply paths"},
    {"probe", (PyCFunction)kw_probe, METH_O, "probe(enable) -> event-loop thread time in native calls since the last call"},
    {"set_partitioned_apply", (PyCFunction)kw_set_partitioned_apply, METH_O,
     "set_partitioned_apply(on) -> previous: batches' apply phase split by pod-cache shard over the decode pool"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_kwcore", "native watch-event decoder", -1, module_methods};

}  // namespace

PyMODINIT_FUNC PyInit__kwcore(void) {
    DecoderType.tp_name = "_kwcore.StreamDecoder";
    DecoderType.tp_basicsize = sizeof(DecoderObject);
    DecoderType.tp_flags = Py_TPFLAGS_DEFAULT;
    DecoderType.tp_doc = "StreamDecoder(environment, state_format='structured')";
    DecoderType.tp_methods = Decoder_methods;
    DecoderType.tp_new = Decoder_new;
    DecoderType.tp_init = (initproc)Decoder_init;
    DecoderType.tp_dealloc = (destructor)Decoder_dealloc;
    if (PyType_Ready(&DecoderType) < 0) return nullptr;
    PyObject* m = PyModule_Create(&moddef);
    if (!m) return nullptr;
    Py_INCREF(&DecoderType);
    PyModule_AddObject(m, "StreamDecoder", (PyObject*)&DecoderType);
    ScannerType.tp_name = "_kwcore.ResponseScanner";
    ScannerType.tp_basicsize = sizeof(ScannerObject);
    ScannerType.tp_flags = Py_TPFLAGS_DEFAULT;
    ScannerType.tp_doc = "ResponseScanner(): incremental HTTP/1.1 response framing";
    ScannerType.tp_methods = Scanner_methods;
    ScannerType.tp_new = Scanner_new;
    ScannerType.tp_dealloc = (destructor)Scanner_dealloc;
    if (PyType_Ready(&ScannerType) < 0) return nullptr;
    Py_INCREF(&ScannerType);
    PyModule_AddObject(m, "ResponseScanner", (PyObject*)&ScannerType);
    if (register_engine(m) < 0 || register_podcache(m) < 0 || register_pipeline(m) < 0 || register_logsink(m) < 0 ||
        register_checkpoint(m) < 0 || register_relist(m) < 0 || register_readerhub(m) < 0 || register_tls13(m) < 0 || register_sinkserver(m) < 0 ||
        register_looplag(m) < 0)
        return nullptr;
    const char* names[6] = {"ADDED", "MODIFIED", "DELETED", "BOOKMARK", "ERROR", "INVALID"};
    for (int i = 0; i < 6; ++i) {
        g_types[i] = PyUnicode_InternFromString(names[i]);
        if (!g_types[i]) return nullptr;
    }
    PyObject* json = PyImport_ImportModule("json");
    if (!json) return nullptr;
    g_json_loads = PyObject_GetAttrString(json, "loads");
    Py_DECREF(json);
    if (!g_json_loads) return nullptr;
#if defined(__x86_64__)
    __builtin_cpu_init();
    Parser::use_avx2 = simd_supported();
    Parser::use_avx512 = avx512_supported();
#endif
    return m;
}
