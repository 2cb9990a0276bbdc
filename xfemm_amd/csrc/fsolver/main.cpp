// fsolver command line: same usage as the reference (cfemm/fsolver/main.cpp):
//   fsolver <problem path without .fem>     -> writes <problem>.ans
// Options (this build): --device N, --keep-mesh (do not delete mesh files).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "fsolver.h"

int main(int argc, char **argv)
{
    xfemm::FSolver theFSolver;
    std::string path;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--device") && i + 1 < argc) theFSolver.device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--keep-mesh")) theFSolver.deleteMeshFiles = false;
        else if (path.empty()) path = argv[i];
        else {
            printf("Too many arguments");
            return 1;
        }
    }
    if (path.empty()) {
        char buf[512];
        printf("Enter fem file name without extension:\n");
        if (!fgets(buf, sizeof buf, stdin)) return 1;
        char *pos = strchr(buf, '\n');
        if (pos) *pos = '\0';
        path = buf;
    }
    if (path.size() > 4 && path.compare(path.size() - 4, 4, ".fem") == 0) path.resize(path.size() - 4);
    theFSolver.PathName = path;
    if (!theFSolver.LoadProblemFile()) {
        theFSolver.WarnMessage("problem loading .fem file\n");
        return 1;
    }
    if (!theFSolver.runSolver(true)) return 2;
    return 0;
}
