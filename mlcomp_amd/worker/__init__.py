"""Worker runtime: task lifecycle, executors, code storage, worker pool and daemon."""
