package ai.foremast.metrics.servlet;

import io.micrometer.core.instrument.Timer;

import javax.servlet.Filter;
import javax.servlet.FilterChain;
import javax.servlet.FilterConfig;
import javax.servlet.ServletException;
import javax.servlet.ServletRequest;
import javax.servlet.ServletResponse;
import javax.servlet.http.HttpServletRequest;
import javax.servlet.http.HttpServletResponse;
import java.io.IOException;
import java.util.Collections;
import java.util.HashMap;
import java.util.Map;

/**
 * Times every request into {@code http.server.requests} with the tags the
 * foremast rules and the downstream-impact graph read: method, uri (the
 * handler's path pattern when Spring MVC set one, else root / NOT_FOUND /
 * REDIRECTION / UNKNOWN, never a raw path: one series per route, not per
 * id), status, outcome, exception, caller (the caller header; {@code
 * callerDefault}, "UNKNOWN" unless set, when absent).  Init parameters
 * (web.xml / FilterRegistration): {@code app}, {@code callerHeader},
 * {@code callerDefault}, {@code initializeForStatuses}, {@code jvmMetrics},
 * and the common-metrics gate's ({@link CommonMetricsGate}).
 * Async requests are recorded when they complete.
 */
public class HttpRequestsFilter implements Filter {

    static final String PATTERN_ATTR = "org.springframework.web.servlet.HandlerMapping.bestMatchingPattern";

    private ForemastMetrics metrics;

    @Override
    public void init(FilterConfig config) {
        Map<String, String> s = new HashMap<>();
        for (String k : Collections.list(config.getInitParameterNames())) {
            s.put(k, config.getInitParameter(k));
        }
        metrics = ForemastMetrics.shared(s);
    }

    @Override
    public void doFilter(ServletRequest req, ServletResponse res, FilterChain chain)
            throws IOException, ServletException {
        if (!(req instanceof HttpServletRequest) || !(res instanceof HttpServletResponse)) {
            chain.doFilter(req, res);
            return;
        }
        HttpServletRequest http = (HttpServletRequest) req;
        HttpServletResponse resp = (HttpServletResponse) res;
        Timer.Sample sample = Timer.start(metrics.registry());
        Throwable failure = null;
        try {
            chain.doFilter(req, res);
        } catch (IOException | ServletException | RuntimeException | Error e) {
            failure = e;
            throw e;
        } finally {
            if (http.isAsyncStarted()) {
                final Timer.Sample s = sample;
                http.getAsyncContext().addListener(new javax.servlet.AsyncListener() {
                    public void onComplete(javax.servlet.AsyncEvent e) { record(s, http, resp, null); }
                    public void onTimeout(javax.servlet.AsyncEvent e) { }
                    public void onError(javax.servlet.AsyncEvent e) { record(s, http, resp, e.getThrowable()); }
                    public void onStartAsync(javax.servlet.AsyncEvent e) { }
                });
            } else {
                record(sample, http, resp, failure);
            }
        }
    }

    void record(Timer.Sample sample, HttpServletRequest req, HttpServletResponse res, Throwable failure) {
        int status = failure != null && res.getStatus() < 400 ? 500 : res.getStatus();
        String caller = req.getHeader(metrics.callerHeader());
        sample.stop(Timer.builder(ForemastMetrics.HTTP_REQUESTS)
                .tags("method", req.getMethod(), "uri", uri(req, status), "status", Integer.toString(status),
                      "outcome", outcome(status),
                      "exception", failure == null ? "None" : failure.getClass().getSimpleName(),
                      "caller", caller == null || caller.trim().isEmpty() ? metrics.callerDefault() : caller.trim())
                .register(metrics.registry()));
    }

    static String uri(HttpServletRequest req, int status) {
        Object pattern = req.getAttribute(PATTERN_ATTR);
        if (pattern != null) {
            return pattern.toString();
        }
        if (status == 404) {
            return "NOT_FOUND";
        }
        if (status >= 300 && status < 400) {
            return "REDIRECTION";
        }
        String path = req.getRequestURI().substring(req.getContextPath().length());
        return path.isEmpty() || "/".equals(path) ? "root" : "UNKNOWN";
    }

    static String outcome(int status) {
        switch (status / 100) {
            case 1: return "INFORMATIONAL";
            case 2: return "SUCCESS";
            case 3: return "REDIRECTION";
            case 4: return "CLIENT_ERROR";
            case 5: return "SERVER_ERROR";
            default: return "UNKNOWN";
        }
    }

    @Override
    public void destroy() {
    }
}
