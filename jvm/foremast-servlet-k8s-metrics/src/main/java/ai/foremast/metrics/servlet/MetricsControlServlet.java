package ai.foremast.metrics.servlet;

import javax.servlet.ServletConfig;
import javax.servlet.http.HttpServlet;
import javax.servlet.http.HttpServletRequest;
import javax.servlet.http.HttpServletResponse;
import java.io.IOException;
import java.util.Collections;
import java.util.HashMap;
import java.util.Map;

/**
 * Runtime enable / disable of a metric: {@code GET|POST <mapping>/enable/<metric>}
 * and {@code <mapping>/disable/<metric>} (the reference's
 * {@code /k8s-metrics/{enable,disable}/{metric}} actuator endpoint,
 * foremast-spring-boot-k8s-metrics-starter/.../K8sMetricsEndpoint.java).
 * Answers {@code true} / {@code false} as JSON (false: runtime actions are
 * off, {@code enableCommonMetricsFilterAction}); 404 for anything else.
 * Map it at {@code /k8s-metrics/*}.
 */
public class MetricsControlServlet extends HttpServlet {

    private ForemastMetrics metrics;

    @Override
    public void init(ServletConfig config) {
        Map<String, String> s = new HashMap<>();
        for (String k : Collections.list(config.getInitParameterNames())) {
            s.put(k, config.getInitParameter(k));
        }
        metrics = ForemastMetrics.shared(s);
    }

    @Override
    protected void doGet(HttpServletRequest req, HttpServletResponse res) throws IOException {
        handle(req, res);
    }

    @Override
    protected void doPost(HttpServletRequest req, HttpServletResponse res) throws IOException {
        handle(req, res);
    }

    private void handle(HttpServletRequest req, HttpServletResponse res) throws IOException {
        String path = req.getPathInfo() == null ? "" : req.getPathInfo();
        String[] parts = path.startsWith("/") ? path.substring(1).split("/", 2) : new String[0];
        if (parts.length != 2 || parts[1].isEmpty() || !("enable".equals(parts[0]) || "disable".equals(parts[0]))) {
            res.sendError(HttpServletResponse.SC_NOT_FOUND);
            return;
        }
        CommonMetricsGate gate = metrics.gate();
        boolean done = "enable".equals(parts[0]) ? gate.enableMetric(parts[1]) : gate.disableMetric(parts[1]);
        res.setContentType("application/json");
        res.getWriter().write(done ? "true" : "false");
    }
}
