// bsgsd_amd — the reference's BSGS daemon (bsgsd.cpp, BSGSD.md) on the MI355X engine.
//
// Options -6 -h -k -n -t -p -i as bsgsd.cpp:390-412, plus -g <ids> (GPUs) and --cpu-build.  The
// tables come from / go to the -S files in the working directory (bsgsd.cpp:179 FLAGSAVEREADFILE = 1)
// and stay resident on the GPUs (one libkhbsgs session) for every request.  Protocol
// (client_handler, bsgsd.cpp:2374-2492): one line "<publickey> <from>:<to>" per connection, tokenised
// on " \t:" after trimming "\t\n\r :" (util.c:67-84); exactly 3 tokens, a valid public key and two
// hex values, else "400 Bad Request"; then a sequential search of [from, to) and one reply — the
// private key in lowercase hex, or "404 Not Found" — and the connection is closed.  One client at a
// time.  Deviation: the reference binds the compile-time port 8080 whatever -p says
// (bsgsd.cpp:1340); here -p is honoured, as BSGSD.md documents.
#include <arpa/inet.h>
#include <getopt.h>
#include <netinet/in.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include "bsgs_host.hpp"
#include "engine.hpp"

using namespace khb;

namespace {

const char* kVersion = "1.0.0 bsgsd_amd (MI355X BSGS engine)";

void menu() {
  printf("\nUsage:\n");
  printf("-h          show this help\n");
  printf("-6          to skip sha256 Checksum on data files\n");
  printf("-t tn       Threads number, must be a positive integer\n");
  printf("-k value    k factor, same as keyhunt\n");
  printf("-n number   Check for N sequential numbers before the random chosen, this only works with -R option\n");
  printf("-i ip       IP Address for listening conections default 127.0.0.1\n");
  printf("-p port     TCP port Number for listening conections\n");
  printf("-g ids      GPU ordinals (default 0)\n");
  printf("--cpu-build build the baby-step tables on the CPU\n");
  printf("--check w   confirm candidates on the host, the gpu, or auto (default host)\n");
  exit(EXIT_FAILURE);
}

bool valid_hex(const char* s) {   // util.c:169-178
  for (; *s; ++s) {
    const char c = *s;
    if (!((c >= '0' && c <= '9') || (c >= 'A' && c <= 'F') || (c >= 'a' && c <= 'f'))) return false;
  }
  return true;
}

// stringtokenizer (util.c:67-84): trim "\t\n\r :" then strtok on " \t:"
std::vector<std::string> tokenize(std::string s) {
  const char* trimset = "\t\n\r :";
  size_t b = s.find_first_not_of(trimset), e = s.find_last_not_of(trimset);
  if (b == std::string::npos) return {};
  s = s.substr(b, e - b + 1);
  std::vector<std::string> out;
  std::vector<char> buf(s.begin(), s.end());
  buf.push_back(0);
  for (char* tok = strtok(buf.data(), " \t:"); tok; tok = strtok(nullptr, " \t:")) out.push_back(tok);
  return out;
}

void send_str(int fd, const std::string& s) {
  if (send(fd, s.data(), s.size(), 0) == -1) printf("Failed to send message to client\n");
}

// client_handler (bsgsd.cpp:2374-2492)
void handle(int fd, Session& S, const Tables& T) {
  char buffer[1024];
  ssize_t n = recv(fd, buffer, sizeof(buffer) - 1, MSG_PEEK);
  if (n <= 0) return;
  const char* nl = (const char*)memchr(buffer, '\n', (size_t)n);
  const size_t line_length = nl ? (size_t)(nl - buffer) + 1 : (size_t)n;
  n = recv(fd, buffer, line_length, 0);
  if (n <= 0) return;
  buffer[n] = 0;
  const std::vector<std::string> t = tokenize(buffer);
  if (t.size() != 3) {
    printf("Invalid input format from client, tokens %i : %s\n", (int)t.size(), buffer);
    send_str(fd, "400 Bad Request");
    return;
  }
  Target tg;
  if (!parse_pubkey_hex(t[0].c_str(), tg.p, tg.compressed, nullptr)) {
    printf("Invalid publickey format from client %s\n", t[0].c_str());
    send_str(fd, "400 Bad Request");
    return;
  }
  if (!(valid_hex(t[1].c_str()) && valid_hex(t[2].c_str()))) {
    printf("Invalid hexadecimal format from client %s:%s\n", t[1].c_str(), t[2].c_str());
    send_str(fd, "400 Bad Request");
    return;
  }
  U256 start, end;
  U256::from_hex(t[1].c_str(), start);
  U256::from_hex(t[2].c_str(), end);
  std::vector<int> found;
  std::vector<U256> keys;
  SearchStats st;
  std::string err;
  SearchCallbacks cb;
  const int rc = S.run({tg}, start, end, cb, found, keys, st, err);
  if (rc) {
    fprintf(stderr, "[E] %s\n", err.c_str());
    return;   // "in case some other error the server will close the Conection without send any error message"
  }
  send_str(fd, found[0] ? keys[0].hex() : std::string("404 Not Found"));
}

}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  signal(SIGPIPE, SIG_IGN);
  printf("[+] Version %s\n", kVersion);
  int kfactor = 1, nthreads = (int)std::thread::hardware_concurrency(), port = 8080;
  bool skip_checksum = false, cpu_build = false;
  const char* str_n = nullptr;
  std::string ip = "127.0.0.1";
  SearchConfig cfg;
  if (nthreads > 16) nthreads = 16;
  static struct option longopts[] = {{"cpu-build", no_argument, nullptr, 1000},
                                     {"check", required_argument, nullptr, 1001},
                                     {nullptr, 0, nullptr, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "6hk:n:t:p:i:g:", longopts, nullptr)) != -1) {
    switch (c) {
      case '6': skip_checksum = true; fprintf(stderr, "[W] Skipping checksums on files\n"); break;
      case 'h': menu(); break;
      case 'k':
        kfactor = (int)strtol(optarg, nullptr, 10);
        if (kfactor <= 0) kfactor = 1;
        printf("[+] K factor %i\n", kfactor);
        break;
      case 'n': str_n = optarg; break;
      case 't':
        nthreads = (int)strtol(optarg, nullptr, 10);
        if (nthreads <= 0) nthreads = 1;
        printf(nthreads > 1 ? "[+] Threads : %u\n" : "[+] Thread : %u\n", nthreads);
        break;
      case 'p':
        port = (int)strtol(optarg, nullptr, 10);
        if (port <= 0 || port > 65535) port = 8080;
        break;
      case 'i': ip = optarg; break;
      case 'g': {
        cfg.devices.clear();
        std::string part;
        for (const char* p = optarg;; ++p) {
          if (*p == ',' || *p == 0) {
            if (!part.empty()) cfg.devices.push_back(atoi(part.c_str()));
            part.clear();
            if (!*p) break;
          } else {
            part.push_back(*p);
          }
        }
        if (cfg.devices.empty()) cfg.devices.push_back(0);
        break;
      }
      case 1000: cpu_build = true; break;
      case 1001:                                    // where candidates are confirmed (engine.hpp check_mode)
        if ((cfg.check_mode = parse_check_mode(optarg)) < 0) {
          fprintf(stderr, "[E] --check: host, gpu or auto\n");
          exit(EXIT_FAILURE);
        }
        break;
      default:
        fprintf(stderr, "[E] Unknow opcion -%c\n", c);
        exit(0);
    }
  }
  printf("[+] Mode BSGS secuential\n");
  Geometry geo;
  std::string err;
  if (!make_geometry(str_n, kfactor, geo, err)) {
    fprintf(stderr, "%s\n", err.c_str());
    exit(EXIT_FAILURE);
  }
  printf("[+] N = 0x%s\n", geo.N.hex().c_str());
  {
    auto mb = [](uint64_t bytes) { return (float)bytes / 1048576.0f; };
    BloomFilter b;
    b.init2(geo.items1, 0.000001);
    printf("[+] Bloom filter for %llu elements : %.2f MB\n", (unsigned long long)geo.m, mb(b.bytes * 256));
    b.init2(geo.items2, 0.000001);
    printf("[+] Bloom filter for %llu elements : %.2f MB\n", (unsigned long long)geo.m2, mb(b.bytes * 256));
    b.init2(geo.items3, 0.000001);
    printf("[+] Bloom filter for %llu elements : %.2f MB\n", (unsigned long long)geo.m3, mb(b.bytes * 256));
    printf("[+] Allocating %.2f MB for %llu bP Points\n", (double)(geo.m3 * 16 / 1048576), (unsigned long long)geo.m3);
  }
  Tables T;
  auto say = [](const std::string& m) { printf("%s", m.c_str()); fflush(stdout); };
  uint32_t have = 0;
  T.prepare(geo);
  if (!T.load_files(".", skip_checksum, have, err, say) ||
      !T.build(geo, nthreads, 4, err, nullptr, have, cpu_build ? -1 : cfg.devices[0]) ||
      (have != kFileAll && !T.save_files(".", have, err, say))) {
    fprintf(stderr, "%s\n", err.c_str());
    exit(EXIT_FAILURE);
  }
  cfg.check_threads = nthreads;
  Session S;
  if (S.open(T, cfg, err)) {
    fprintf(stderr, "[E] %s\n", err.c_str());
    exit(EXIT_FAILURE);
  }
  const int server_fd = socket(AF_INET, SOCK_STREAM, 0);
  if (server_fd < 0) { perror("socket failed"); exit(EXIT_FAILURE); }
  int opt = 1;
  if (setsockopt(server_fd, SOL_SOCKET, SO_REUSEADDR, &opt, sizeof(opt))) {
    perror("setsockopt SO_REUSEADDR failed");
    exit(EXIT_FAILURE);
  }
  sockaddr_in address{};
  address.sin_family = AF_INET;
  address.sin_addr.s_addr = inet_addr(ip.c_str());
  address.sin_port = htons((uint16_t)port);
  if (bind(server_fd, (sockaddr*)&address, sizeof(address)) < 0) { perror("bind failed"); exit(EXIT_FAILURE); }
  printf("[+] Listening in %s:%i\n", ip.c_str(), port);
  if (listen(server_fd, 3) < 0) { perror("listen failed"); exit(EXIT_FAILURE); }
  for (;;) {
    socklen_t addrlen = sizeof(address);
    const int client_fd = accept(server_fd, (sockaddr*)&address, &addrlen);
    if (client_fd < 0) { perror("accept failed"); exit(EXIT_FAILURE); }
    char client_ip[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &address.sin_addr, client_ip, INET_ADDRSTRLEN);
    const int client_port = ntohs(address.sin_port);
    printf("[+] Accepting incoming conection from %s:%i\n", client_ip, client_port);
    handle(client_fd, S, T);
    close(client_fd);
    printf("[+] Closing conection from %s:%i\n", client_ip, client_port);
  }
}
