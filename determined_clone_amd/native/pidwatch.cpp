// dca-pidwatch: worker-failure detection for multi-process launches (native replacement of the
// reference's harness/determined/exec/pid_server.py + pid_client.py + ipc.PIDServer/PIDClient).
//
//   dca-pidwatch server [--on-fail SIG|WAIT] [--on-exit SIG|WAIT] [--grace-period S]
//                       [--signal-children] ADDR NUM_WORKERS -- CMD ARGS...
//   dca-pidwatch client ADDR -- CMD ARGS...
//
// ADDR is a unix-socket path, a TCP port ("29500") or "host:port". The server runs CMD (the launch
// layer, e.g. torch.distributed.run or an ssh fan-out) as a child in its own process group and
// accepts NUM_WORKERS client connections. Each client reports "<pid>\n", runs its worker, sends a
// keepalive byte 'k' every second and 'q' when the worker exits with status 0. A connection that
// closes without 'q' (crash, OOM kill, lost node) is a worker failure: the server sends --on-fail
// (default SIGTERM) to the launch layer's process group and to every known worker pid, escalates to
// SIGKILL after --grace-period seconds, and exits non-zero. When the launch layer exits by itself,
// --on-exit (default WAIT) decides whether stragglers are signalled. Exit codes: the launch layer's
// status, 70 on a detected worker failure.
#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace {

constexpr int kWorkerFailed = 70;

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// "WAIT" -> 0, else signal number (SIGTERM / TERM / 15)
int parse_action(const std::string& v) {
  std::string u;
  for (char c : v) u += static_cast<char>(toupper(c));
  if (u == "WAIT") return 0;
  if (u.rfind("SIG", 0) == 0) u = u.substr(3);
  static const std::map<std::string, int> names = {
      {"TERM", SIGTERM}, {"KILL", SIGKILL}, {"INT", SIGINT}, {"HUP", SIGHUP},
      {"QUIT", SIGQUIT}, {"USR1", SIGUSR1}, {"USR2", SIGUSR2}};
  auto it = names.find(u);
  if (it != names.end()) return it->second;
  char* end = nullptr;
  long n = strtol(u.c_str(), &end, 10);
  if (end && *end == 0 && n > 0 && n < 65) return static_cast<int>(n);
  fprintf(stderr, "dca-pidwatch: invalid action '%s' (signal name or WAIT)\n", v.c_str());
  exit(2);
}

struct Addr {
  bool unix_sock = false;
  std::string path, host;
  int port = 0;
};

Addr parse_addr(const std::string& a) {
  Addr r;
  bool digits = !a.empty();
  for (char c : a) digits &= (c >= '0' && c <= '9');
  if (digits) {
    r.port = atoi(a.c_str());
    r.host = "127.0.0.1";
    return r;
  }
  auto colon = a.rfind(':');
  if (colon != std::string::npos && a.find('/') == std::string::npos) {
    r.host = a.substr(0, colon);
    r.port = atoi(a.substr(colon + 1).c_str());
    return r;
  }
  r.unix_sock = true;
  r.path = a;
  return r;
}

int make_listener(const Addr& a, int backlog) {
  int fd;
  if (a.unix_sock) {
    fd = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un sa{};
    sa.sun_family = AF_UNIX;
    if (a.path.size() >= sizeof(sa.sun_path)) { fprintf(stderr, "socket path too long\n"); exit(2); }
    strcpy(sa.sun_path, a.path.c_str());
    unlink(a.path.c_str());
    if (bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) { perror("bind"); exit(2); }
  } else {
    fd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(a.port));
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa)) != 0) { perror("bind"); exit(2); }
  }
  if (listen(fd, backlog) != 0) { perror("listen"); exit(2); }
  return fd;
}

int connect_to(const Addr& a, double timeout_s) {
  const double t0 = now_s();
  while (true) {
    int fd;
    int rc;
    if (a.unix_sock) {
      fd = socket(AF_UNIX, SOCK_STREAM, 0);
      sockaddr_un sa{};
      sa.sun_family = AF_UNIX;
      strncpy(sa.sun_path, a.path.c_str(), sizeof(sa.sun_path) - 1);
      rc = connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof(sa));
    } else {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      const std::string port = std::to_string(a.port);
      if (getaddrinfo(a.host.c_str(), port.c_str(), &hints, &res) != 0 || !res) {
        fprintf(stderr, "dca-pidwatch: cannot resolve %s\n", a.host.c_str());
        exit(2);
      }
      fd = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      rc = connect(fd, res->ai_addr, res->ai_addrlen);
      freeaddrinfo(res);
    }
    if (rc == 0) return fd;
    close(fd);
    if (now_s() - t0 > timeout_s) {
      fprintf(stderr, "dca-pidwatch client: could not reach pid server: %s\n", strerror(errno));
      exit(2);
    }
    usleep(100 * 1000);
  }
}

pid_t spawn(const std::vector<std::string>& cmd, bool new_group) {
  pid_t pid = fork();
  if (pid < 0) { perror("fork"); exit(2); }
  if (pid == 0) {
    if (new_group) setpgid(0, 0);
    std::vector<char*> argv;
    for (auto& s : cmd) argv.push_back(const_cast<char*>(s.c_str()));
    argv.push_back(nullptr);
    execvp(argv[0], argv.data());
    fprintf(stderr, "dca-pidwatch: exec %s failed: %s\n", argv[0], strerror(errno));
    _exit(127);
  }
  if (new_group) setpgid(pid, pid);
  return pid;
}

int status_code(int st) {
  if (WIFEXITED(st)) return WEXITSTATUS(st);
  if (WIFSIGNALED(st)) return 128 + WTERMSIG(st);
  return 1;
}

void signal_all(pid_t child, const std::set<int>& pids, int sig, bool children) {
  if (child > 0) kill(children ? -child : child, sig);
  for (int p : pids) kill(p, sig);
}

// ------------------------------------------------------------------------------------- server
int run_server(int on_fail, int on_exit, double grace, bool signal_children, const std::string& addr,
               int num_workers, const std::vector<std::string>& cmd) {
  const Addr a = parse_addr(addr);
  int lfd = make_listener(a, num_workers);
  signal(SIGPIPE, SIG_IGN);
  pid_t child = spawn(cmd, true);
  std::map<int, int> conn_pid;      // fd -> worker pid (-1 until the pid line arrived)
  std::map<int, std::string> bufs;  // partial pid lines
  std::set<int> pids, graceful;
  int accepted = 0;
  bool failed = false;
  int child_status = -1;
  double fail_time = 0;
  while (true) {
    // reap the launch layer
    if (child_status < 0) {
      int st;
      pid_t r = waitpid(child, &st, WNOHANG);
      if (r == child) {
        child_status = status_code(st);
        if (!failed && on_exit) signal_all(0, pids, on_exit, false);
        if (failed || conn_pid.empty()) break;
      }
    } else if (conn_pid.empty() || failed) {
      break;
    }
    if (failed && child_status < 0 && now_s() - fail_time > grace) {
      signal_all(child, pids, SIGKILL, true);
    }
    std::vector<pollfd> fds;
    if (lfd >= 0) fds.push_back({lfd, POLLIN, 0});
    for (auto& kv : conn_pid) fds.push_back({kv.first, POLLIN, 0});
    int n = poll(fds.data(), fds.size(), 200);
    if (n < 0 && errno != EINTR) { perror("poll"); break; }
    for (auto& p : fds) {
      if (!(p.revents & (POLLIN | POLLHUP | POLLERR))) continue;
      if (p.fd == lfd) {
        int c = accept(lfd, nullptr, nullptr);
        if (c < 0) continue;
        conn_pid[c] = -1;
        if (++accepted == num_workers) {
          close(lfd);
          lfd = -1;
          if (a.unix_sock) unlink(a.path.c_str());
        }
        continue;
      }
      char buf[256];
      ssize_t k = recv(p.fd, buf, sizeof(buf), 0);
      int& wpid = conn_pid[p.fd];
      if (k > 0) {
        std::string s(buf, buf + k);
        if (wpid < 0) {
          bufs[p.fd] += s;
          auto nl = bufs[p.fd].find('\n');
          if (nl == std::string::npos) continue;
          wpid = atoi(bufs[p.fd].substr(0, nl).c_str());
          pids.insert(wpid);
          s = bufs[p.fd].substr(nl + 1);
          bufs.erase(p.fd);
          if (s.empty()) continue;
        }
        if (s.back() == 'q') graceful.insert(wpid);
        continue;  // 'k' keepalives (or 'q' followed by EOF later)
      }
      // EOF / error: the worker is gone. Copy the pid out before erase(): wpid refers into the
      // map node (use-after-free found by the ASan build, tests/test_native_sanitizers.py).
      const int gone = wpid;
      const bool ok = gone >= 0 && graceful.count(gone);
      close(p.fd);
      conn_pid.erase(p.fd);
      if (!ok && !failed) {
        failed = true;
        fail_time = now_s();
        fprintf(stderr, "dca-pidwatch: worker %d exited without a graceful shutdown; "
                "stopping the job\n", gone);
        if (on_fail) signal_all(child, pids, on_fail, signal_children);
      }
    }
  }
  if (lfd >= 0) {
    close(lfd);
    if (a.unix_sock) unlink(a.path.c_str());
  }
  if (child_status < 0) {
    int st;
    waitpid(child, &st, 0);
    child_status = status_code(st);
  }
  if (failed) return kWorkerFailed;
  return child_status;
}

// ------------------------------------------------------------------------------------- client
int run_client(const std::string& addr, const std::vector<std::string>& cmd) {
  const Addr a = parse_addr(addr);
  signal(SIGPIPE, SIG_IGN);
  int fd = connect_to(a, 60.0);
  pid_t child = spawn(cmd, false);
  const std::string line = std::to_string(child) + "\n";
  (void)!write(fd, line.data(), line.size());
  int st = 0;
  while (true) {
    pid_t r = waitpid(child, &st, WNOHANG);
    if (r == child) break;
    if (write(fd, "k", 1) < 0) {
      // the server is gone: the job is being torn down
      kill(child, SIGTERM);
      waitpid(child, &st, 0);
      break;
    }
    for (int i = 0; i < 10; ++i) {
      usleep(100 * 1000);
      if (waitpid(child, &st, WNOHANG) == child) goto done;
    }
  }
done:
  const int code = status_code(st);
  if (code == 0) (void)!write(fd, "q", 1);
  close(fd);
  return code;
}

void usage() {
  fprintf(stderr,
          "usage: dca-pidwatch server [--on-fail SIG|WAIT] [--on-exit SIG|WAIT] [--grace-period S]\n"
          "                           [--signal-children] ADDR NUM_WORKERS -- CMD...\n"
          "       dca-pidwatch client ADDR -- CMD...\n");
  exit(2);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) usage();
  const std::string mode = argv[1];
  std::vector<std::string> pos, cmd;
  int on_fail = SIGTERM, on_exit = 0;
  double grace = 3.0;
  bool signal_children = false;
  int i = 2;
  for (; i < argc; ++i) {
    const std::string s = argv[i];
    if (s == "--") { ++i; break; }
    if (s == "--on-fail" || s == "-x") on_fail = parse_action(argv[++i]);
    else if (s == "--on-exit" || s == "-e") on_exit = parse_action(argv[++i]);
    else if (s == "--grace-period") grace = atof(argv[++i]);
    else if (s == "--signal-children") signal_children = true;
    else pos.push_back(s);
  }
  for (; i < argc; ++i) cmd.push_back(argv[i]);
  if (cmd.empty()) usage();
  if (mode == "server") {
    if (pos.size() != 2) usage();
    return run_server(on_fail, on_exit, grace, signal_children, pos[0], atoi(pos[1].c_str()), cmd);
  }
  if (mode == "client") {
    if (pos.size() != 1) usage();
    return run_client(pos[0], cmd);
  }
  usage();
  return 2;
}
