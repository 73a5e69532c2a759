// Rank-prefixed leveled logging to stderr. stdout carries results only (byte-compatible with
// main.c:204); the reference printed its errors to stdout (cudaFunctions.cu:20,30).
#pragma once

#include <cstdarg>
#include <string>

namespace moc {

enum class LogLevel : int { Error = 0, Warn = 1, Info = 2, Debug = 3 };

void log_set_level(LogLevel lvl);
void log_set_level(const std::string& name);  // error|warn|info|debug
void log_set_rank(int rank);
LogLevel log_level();
void logf(LogLevel lvl, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define MOC_LOG_ERROR(...) ::moc::logf(::moc::LogLevel::Error, __VA_ARGS__)
#define MOC_LOG_WARN(...) ::moc::logf(::moc::LogLevel::Warn, __VA_ARGS__)
#define MOC_LOG_INFO(...) ::moc::logf(::moc::LogLevel::Info, __VA_ARGS__)
#define MOC_LOG_DEBUG(...) ::moc::logf(::moc::LogLevel::Debug, __VA_ARGS__)

}  // namespace moc
