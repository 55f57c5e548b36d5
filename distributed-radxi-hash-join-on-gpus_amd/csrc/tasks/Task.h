// Unit of work + type tag, as /root/reference/tasks/Task.h:10-30.  On the
// device a task's execute() ENQUEUES its kernels on the engine's streams; the
// HashJoin operator only synchronises where a host decision needs data.
#pragma once

enum task_type_t { TASK_HISTOGRAM, TASK_NET_PARTITION, TASK_PARTITION, TASK_BUILD_PROBE };

namespace hpcjoin {
namespace tasks {

class Task {
 public:
  virtual ~Task() {}
  virtual void execute() = 0;
  virtual task_type_t getType() = 0;
};

}  // namespace tasks
}  // namespace hpcjoin
